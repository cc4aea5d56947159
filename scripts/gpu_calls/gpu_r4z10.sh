#!/bin/bash
# round 4 (call Z10): generation GPU tests after moving the decode-graph registry out of the module.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
PT="python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $PT tests/test_generate_gpu.py tests/test_generate.py > gpurun_out/z10_gen.log 2>&1; rc=$?
echo "=== z10_gen rc=$rc $(grep -E 'passed|failed' gpurun_out/z10_gen.log | tail -1)"; grep FAILED gpurun_out/z10_gen.log | head
exit $rc
