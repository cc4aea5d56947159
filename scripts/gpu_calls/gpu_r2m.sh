#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ops_gpu.py -k "gemm" > gpurun_out/m_tests.log 2>&1
for s in "8192 8192 8192 nt" "65536 768 3072 nt" "65536 768 50304 nn" "65536 2304 768 nt"; do
  for r in 1 2; do timeout -k 10 60 python3 scripts/gemm_one.py $s --cfg 9 --iters 20 >> gpurun_out/m_gemm.log 2>&1; done
done
for r in 1 2; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/m_b.log 2>&1; tail -1 gpurun_out/m_b.log | cut -c1-200 >> gpurun_out/m_bench.log; done
