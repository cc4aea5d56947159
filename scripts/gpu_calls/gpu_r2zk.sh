#!/bin/bash
# GPT-2-small per-GPU micro-batch sweep (graph mode, 1 GPU): throughput vs micro-batch (info; the bench default stays 64).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2zk
set -e
for b in 32 64 96 128; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch $b > gpurun_out/r2zk/b$b.log 2>&1
done
