#!/bin/bash
# LN-backward grid size A/B end to end (the column-sum pass reads one partial row per block): 8192 (default) vs 4096 vs 2048 waves.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2zn
set -e
for r in 1 2; do
  for w in 8192 4096 2048; do
    REPLICANN_LN_BWD_WAVES=$w timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2zn/w${w}_$r.log 2>&1
  done
done
