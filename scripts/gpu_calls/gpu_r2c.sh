#!/bin/bash
# Round-2 GPU call: attention head sizes 32/128 (MFMA) tests + determinism + refblock graph/dropout,
# then attention A/B timings per head size.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
set -e
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_ops_gpu.py -k "attention" tests/test_determinism_gpu.py tests/test_reference_parity_gpu.py \
  > gpurun_out/attn_tests.log 2>&1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_convergence_gpu.py -k "refblock or graph_replay" > gpurun_out/refblock.log 2>&1
for D in 64 32 128; do
  timeout -k 10 200 python scripts/attn_ab.py 16 --D $D --fwd 3 --bwd 1 >> gpurun_out/attn_ab_d.log 2>&1
done
