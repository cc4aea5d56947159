#!/bin/bash
# Deterministic generic-head attention backward: attention GPU tests + determinism suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
set -e
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ops_gpu.py tests/test_determinism_gpu.py tests/test_reference_parity_gpu.py -k "attention or attn or Attention or parity or bitwise" > gpurun_out/r2zl_tests.log 2>&1
