#!/bin/bash
# spread (deferred per-quadrant) epilogue in cfg 9: GEMM tests, per-shape A/B, bench A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ops_gpu.py tests/test_determinism_gpu.py tests/test_convergence_gpu.py > gpurun_out/spread_tests.log 2>&1
for s in "8192 8192 8192 nt" "65536 2304 768 nt" "65536 768 3072 nt" "65536 3072 768 nt --act 5 --bias" "65536 768 768 nn" "2304 768 65536 tn --split 4"; do
  for e in 0 1 0 1; do
    REPLICANN_GEMM_SPREAD=$e timeout -k 10 60 python3 scripts/gemm_one.py $s --cfg 9 --iters 20 | sed "s/^/spread=$e /" >> gpurun_out/spread_ab.log 2>&1
  done
done
for e in 0 1 0 1; do
  REPLICANN_GEMM_SPREAD=$e timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bs_$e.log 2>&1
  echo "spread=$e $(tail -1 gpurun_out/bs_$e.log | cut -c1-220)" >> gpurun_out/spread_bench.log
done
