#!/bin/bash
# xent v2: GPU tests (CE + fp8), A/B at the GPT-2-small shape, headline bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
set -e
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "xent or cross_entropy or fp8" > gpurun_out/r2s_tests.log 2>&1
timeout -k 10 300 python scripts/xent_ab.py > gpurun_out/r2s_xent_ab.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/r2s_bench.log 2>&1
