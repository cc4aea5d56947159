#!/bin/bash
# round 6 call X: ViT-B/16 step breakdown on the current tree (kernel trace, 3 steps) + PMC of the resident attention kernels
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
M=vit-b16
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_brk_$M -o run -- python3 bench.py --model $M --steps 3 --warmup 2 > gpurun_out/r6x_brk_$M.log 2>&1 || { echo "prof $M failed"; tail -3 gpurun_out/r6x_brk_$M.log; exit 1; }
python3 scripts/prof_steps.py gpurun_out/prof_brk_$M/run_kernel_trace.csv --steps 3 > gpurun_out/r6x_steps_$M.txt 2>&1
rm -rf gpurun_out/prof_brk_$M
head -16 gpurun_out/r6x_steps_$M.txt | cut -c1-150
timeout -k 10 200 bash scripts/pmc_attn.sh "512 --T 197 --noncausal --rounds 1" vitres2 && \
python3 scripts/pmc_summary.py gpurun_out/pmc_attn/vitres2*_counter_collection.csv --match attn > gpurun_out/r6x_pmc.txt 2>&1; rc=$?
cut -c1-330 gpurun_out/r6x_pmc.txt; exit $rc
