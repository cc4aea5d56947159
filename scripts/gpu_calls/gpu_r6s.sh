#!/bin/bash
# round 6 call S: resident attention backward with opaque LDS addressing + fragment prefetch: numerics + timing
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "attention or attn" > gpurun_out/r6s_tests.log 2>&1; rc=$?
grep -E "FAIL|passed|failed" gpurun_out/r6s_tests.log | tail -12; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 scripts/attn_ab.py 512 --T 197 --noncausal --rounds 5 > gpurun_out/r6s_ab.log 2>&1; rc=$?
cat gpurun_out/r6s_ab.log | cut -c1-300; exit $rc
