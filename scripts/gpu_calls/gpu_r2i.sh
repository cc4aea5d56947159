#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_ops_gpu.py -k "attention" > gpurun_out/v3_tests.log 2>&1
timeout -k 10 200 python scripts/attn_ab.py 64 --fwd 3,4 --bwd 1 --rounds 4 > gpurun_out/v3_ab.log 2>&1
timeout -k 10 200 python scripts/attn_ab.py 16 --fwd 3,4 --bwd 1 --rounds 4 >> gpurun_out/v3_ab.log 2>&1
for s in "8192 8192 8192 nt" "65536 2304 768 nt" "65536 768 3072 nt" "65536 768 50304 nn"; do
  for c in 9 91 92 94 98 9; do
    timeout -k 10 60 python3 scripts/gemm_one.py $s --cfg $c --iters 20 >> gpurun_out/abl.log 2>&1
  done
done
