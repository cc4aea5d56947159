#!/bin/bash
# round 6 call AF: resident attention edge cases (T = 1, Tq > Tk tiny, causal with offsets)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "resident" > gpurun_out/r6af_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|passed|failed" gpurun_out/r6af_tests.log | tail -14; exit $rc
