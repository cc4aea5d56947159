#!/bin/bash
# round 6 call F: PMC of the 32x32x16 attention kernels vs the 16x16x32 ones (GPT-2-small shapes, causal)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
REPLICANN_ATTN32=1 bash scripts/pmc_attn.sh "64 --rounds 1" a32 || exit 1
REPLICANN_ATTN32=0 bash scripts/pmc_attn.sh "64 --rounds 1" a16 || exit 1
python3 scripts/pmc_summary.py gpurun_out/pmc_attn/a32*_counter_collection.csv --match attn > gpurun_out/r6f_pmc.txt 2>&1
python3 scripts/pmc_summary.py gpurun_out/pmc_attn/a16*_counter_collection.csv --match attn >> gpurun_out/r6f_pmc.txt 2>&1
cat gpurun_out/r6f_pmc.txt
