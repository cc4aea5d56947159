#!/bin/bash
# round 3: fused-dQ attention backward — numerics/determinism, then A/B timing at GPT-2-small shapes
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_determinism_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "attention" > gpurun_out/attn_test.log 2>&1
rc=$?; tail -3 gpurun_out/attn_test.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python scripts/attn_ab.py 64 --fwd 3 --bwd 2,3 --rounds 3 > gpurun_out/attn_ab.jsonl 2>&1; rc=$?
cat gpurun_out/attn_ab.jsonl | grep -v amdgpu.ids; exit $rc
