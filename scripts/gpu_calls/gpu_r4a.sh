#!/bin/bash
# round 4 (call A, validation): tr_b8 semantics probe, fp8 weight-gradient kernel, staged GEMM
# epilogue + parameter-gradient reference parity, the whole GPU tier, smoke
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -E "passed|failed|smoke ok" gpurun_out/$n.log | tail -1
  return $rc
}
PT="python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider"
step tr8_probe 30 ./scripts/dev/tr8_probe; [ $? -ge 124 ] && exit 1
head -20 gpurun_out/tr8_probe.log
step t_fp8w 300 $PT tests/test_fp8_wgrad_gpu.py; [ $? -ge 124 ] && exit 1
grep -E "^E |Error" gpurun_out/t_fp8w.log | head -20
step t_staged 300 $PT tests/test_gemm_staged_gpu.py tests/test_reference_parity_gpu.py; [ $? -ge 124 ] && exit 1
grep -E "^E |FAILED" gpurun_out/t_staged.log | head -20
step gpu_all 900 $PT tests -m gpu --deselect tests/test_fp8_wgrad_gpu.py; [ $? -ge 124 ] && exit 1
grep -E "FAILED" gpurun_out/gpu_all.log | head -20
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
exit 0
