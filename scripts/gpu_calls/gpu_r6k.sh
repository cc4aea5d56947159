#!/bin/bash
# round 6 call K: full GPU test tier + smoke on this round's tree, then the 1-GPU comm proxy (an 8-rank ring's
# traffic emulated beside the step; verdict r5 item 7) against the plain step, eager form, alternating
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r6k_gpu_tests.log 2>&1; rc=$?
echo "=== gpu tests rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/r6k_gpu_tests.log | tail -6
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6k_smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/r6k_smoke.log; exit 1; }
tail -1 gpurun_out/r6k_smoke.log
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc $(grep -v amdgpu.ids gpurun_out/$n.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')"
  return $rc
}
for r in 1 2; do
  step r6k_plain_eager_$r 300 python bench.py --steps 10 --warmup 3 --graph off || exit 1
  step r6k_proxy_eager_$r 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy --graph off || exit 1
done
exit 0
