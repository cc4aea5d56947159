#!/bin/bash
# round 4 (call A, validation): fp8 weight-gradient kernel, staged GEMM epilogue + parameter-gradient
# reference parity, test_ops_gpu.py alone (an illegal address surfaced there in the previous call,
# after the other files had run), then the rest of the GPU tier, smoke.  Any HIP fault ends the call.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -E "passed|failed|smoke ok" gpurun_out/$n.log | tail -1
  if grep -q "illegal memory access\|hipErrorIllegalAddress\|HSA_STATUS_ERROR\|Memory access fault" gpurun_out/$n.log; then
    echo "GPU FAULT in $n: stopping"; grep -n -m5 "illegal\|fault\|Error" gpurun_out/$n.log; exit 2
  fi
  [ $rc -ge 124 ] && exit 1
  return 0
}
PT="python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider"
step t_fp8w 300 $PT tests/test_fp8_wgrad_gpu.py
grep -E "^E  |FAILED" gpurun_out/t_fp8w.log | head -20
step t_staged 300 $PT tests/test_gemm_staged_gpu.py tests/test_reference_parity_gpu.py
grep -E "^E  |FAILED" gpurun_out/t_staged.log | head -20
step t_ops 600 $PT -x tests/test_ops_gpu.py
grep -E "^E  |FAILED" gpurun_out/t_ops.log | head -20
step gpu_rest 900 $PT tests -m gpu --deselect tests/test_fp8_wgrad_gpu.py --deselect tests/test_ops_gpu.py
grep -E "FAILED" gpurun_out/gpu_rest.log | head -20
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
exit 0
