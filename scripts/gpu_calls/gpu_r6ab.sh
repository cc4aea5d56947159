#!/bin/bash
# round 6 call AB: memory-side traffic of the GPT-2-small (B64 causal T1024) and ViT (B512 T197) attention kernels
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/pmc_mem; export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/pmc_mem -o gpt_a -- python3 scripts/attn_ab.py 64 --rounds 1 > /dev/null 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_mem -o gpt_b -- python3 scripts/attn_ab.py 64 --rounds 1 > /dev/null 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/pmc_mem -o vit_a -- python3 scripts/attn_ab.py 512 --T 197 --noncausal --rounds 1 > /dev/null 2>&1 && \
python3 scripts/pmc_summary.py gpurun_out/pmc_mem/*_counter_collection.csv --match attn > gpurun_out/r6ab_pmc.txt 2>&1; rc=$?
cut -c1-400 gpurun_out/r6ab_pmc.txt; exit $rc
