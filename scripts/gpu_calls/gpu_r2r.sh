#!/bin/bash
# fp8 forward GEMM on the persistent kernel: fp8 GPU tests, kernel A/B, GPT-2-medium bf16 vs fp8 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
set -e
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "fp8" > gpurun_out/r2r_fp8_tests.log 2>&1
timeout -k 10 300 python scripts/fp8_ab.py > gpurun_out/r2r_fp8_ab.log 2>&1
timeout -k 10 400 python bench.py --model gpt2-medium-fp8 --steps 10 --warmup 3 > gpurun_out/r2r_bench_med_fp8.log 2>&1
timeout -k 10 400 python bench.py --model gpt2-medium --steps 10 --warmup 3 > gpurun_out/r2r_bench_med_bf16.log 2>&1
