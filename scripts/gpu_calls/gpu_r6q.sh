#!/bin/bash
# round 6 call Q: whole-head resident attention forward (T <= 256): attention numerics + ViT / GPT-2 timing
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "attention or attn" > gpurun_out/r6q_tests.log 2>&1; rc=$?
grep -E "FAIL|passed|failed" gpurun_out/r6q_tests.log | tail -12; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 scripts/attn_ab.py 512 --T 197 --noncausal --rounds 5 > gpurun_out/r6q_ab.log 2>&1 && \
timeout -k 10 200 python3 scripts/attn_ab.py 64 --rounds 3 >> gpurun_out/r6q_ab.log 2>&1 && \
timeout -k 10 200 python3 scripts/attn_ab.py 512 --T 256 --rounds 3 >> gpurun_out/r6q_ab.log 2>&1; rc=$?
cat gpurun_out/r6q_ab.log | cut -c1-300; exit $rc
