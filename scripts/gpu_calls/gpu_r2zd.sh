#!/bin/bash
# Autotuner variance: the headline bench 4x on one box (separate processes), tuning tables kept.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2zd
set -e
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2zd/bench_$i.log 2>&1
  cp gpurun_out/gemm_tuning_gpt2-small.json gpurun_out/r2zd/tuning_$i.json
done
