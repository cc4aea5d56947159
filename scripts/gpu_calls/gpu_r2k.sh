#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
set -e
for s in "8192 8192 8192 nt" "65536 768 3072 nt" "65536 768 50304 nn"; do
  for c in 9 91 106 9 91 106; do
    timeout -k 10 60 python3 scripts/gemm_one.py $s --cfg $c --iters 20 >> gpurun_out/abl2.log 2>&1
  done
done
