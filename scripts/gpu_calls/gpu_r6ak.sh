#!/bin/bash
# round 6 call AK: shipped-binary check at the end of the round: smoke + attention / GEMM GPU tests + default bench
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6ak_smoke.log 2>&1 || { tail -5 gpurun_out/r6ak_smoke.log; exit 1; }
tail -1 gpurun_out/r6ak_smoke.log
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py > gpurun_out/r6ak_tests.log 2>&1; rc=$?
tail -1 gpurun_out/r6ak_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r6ak_bench.log 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r6ak_bench.log | tr '\n' ' '
