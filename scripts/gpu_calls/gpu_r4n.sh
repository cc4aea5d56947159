#!/bin/bash
# round 4 (call N): PMC counters of every kernel in the GPT-2-small step at HEAD (MFMA busy, wait split,
# LDS conflicts, VALU / MFMA instruction mix, HBM fetch) — 3 rocprofv3 passes of 2 steps each.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 bash scripts/pmc_step.sh "--steps 2 --warmup 1" gpt2s > gpurun_out/n_pmc.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/n_pmc.log; exit 1; }
python scripts/pmc_summary.py gpurun_out/pmc_step/gpt2s*_counter_collection.csv > gpurun_out/pmc_step_summary.txt 2>&1
head -60 gpurun_out/pmc_step_summary.txt | cut -c1-260
exit 0
