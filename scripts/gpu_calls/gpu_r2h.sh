#!/bin/bash
# cfg 9 ablations (timing only, wrong outputs): 91 no DMA, 92 no vmcnt waits, 94 no epilogue, 98 DMA between k-steps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
set -e
for s in "8192 8192 8192 nt" "65536 2304 768 nt" "65536 768 3072 nt" "65536 768 50304 nn"; do
  for c in 9 91 92 94 98 9; do
    timeout -k 10 60 python3 scripts/gemm_one.py $s --cfg $c --iters 20 >> gpurun_out/abl.log 2>&1
  done
done
