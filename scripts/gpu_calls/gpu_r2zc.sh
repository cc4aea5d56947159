#!/bin/bash
# CE dgrad scale folded into the GEMM epilogue: model/loss GPU tests + headline bench x2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
set -e
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_models.py tests/test_convergence_gpu.py tests/test_ops_gpu.py -k "gpt2 or cross or xent or lm or trajectory or graph" > gpurun_out/r2zc_tests.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2zc_bench1.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2zc_bench2.log 2>&1
