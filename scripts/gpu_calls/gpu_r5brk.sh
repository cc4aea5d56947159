#!/bin/bash
# round 5: step breakdowns of the final tree — GPT-2-medium-fp8 (final fp8 defaults) and GPT-2-small (headline)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for M in gpt2-medium-fp8 gpt2-small; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_brk_$M -o run -- python3 bench.py --model $M --steps 3 --warmup 2 > gpurun_out/r5brk_$M.log 2>&1 || { echo "prof $M failed"; exit 1; }
  python scripts/prof_steps.py gpurun_out/prof_brk_$M/run_kernel_trace.csv --steps 3 > gpurun_out/r5brk_steps_$M.txt 2>&1
  rm -rf gpurun_out/prof_brk_$M
  echo "== $M"; head -26 gpurun_out/r5brk_steps_$M.txt | cut -c1-150
done
