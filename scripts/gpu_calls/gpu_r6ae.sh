#!/bin/bash
# round 6 call AE: final-tree step breakdowns (kernel trace, 3 steps) for GPT-2-small and GPT-2-medium fp8
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for M in gpt2-small gpt2-medium-fp8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_brk_$M -o run -- python3 bench.py --model $M --steps 3 --warmup 2 > gpurun_out/r6ae_brk_$M.log 2>&1 || { echo "prof $M failed"; tail -3 gpurun_out/r6ae_brk_$M.log; exit 1; }
  python3 scripts/prof_steps.py gpurun_out/prof_brk_$M/run_kernel_trace.csv --steps 3 > gpurun_out/r6ae_steps_$M.txt 2>&1
  rm -rf gpurun_out/prof_brk_$M
  echo "== $M"; head -14 gpurun_out/r6ae_steps_$M.txt | cut -c1-150
done
