#!/bin/bash
# Deterministic (fixed-point) embedding backward + determinism suite + GPT-2 bench with and without the mode.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
set -e
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_determinism_gpu.py tests/test_models.py -k "embedding or bitwise or gpt2 or deterministic" > gpurun_out/r2zm_tests.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r2zm_bench.log 2>&1
REPLICANN_DETERMINISTIC=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r2zm_bench_det.log 2>&1
