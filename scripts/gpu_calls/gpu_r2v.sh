#!/bin/bash
# fp8 blocks fed by the LayerNorm kernel (c_attn / c_fc in e4m3, projections bf16): GPU tests + GPT-2-medium bf16 vs fp8 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
set -e
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_models.py -k "fp8 or layernorm" > gpurun_out/r2v_tests.log 2>&1
timeout -k 10 400 python bench.py --model gpt2-medium-fp8 --steps 10 --warmup 3 > gpurun_out/r2v_bench_med_fp8.log 2>&1
timeout -k 10 400 python bench.py --model gpt2-medium --steps 10 --warmup 3 > gpurun_out/r2v_bench_med_bf16.log 2>&1
