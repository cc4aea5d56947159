#!/bin/bash
# round 3 (session 2): DDP collective schedule under the 8-GPU comm proxy: eager (issue when ready) vs
# window (beside the next attention backward) vs end (after the backward); fp32 and rsag
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | grep -o '"ms_per_step": [0-9.]*' | tail -1; grep -E "passed|failed" gpurun_out/$n.log | tail -1
  return $rc
}
step commtest 600 python -u -m pytest tests/test_comm_gpu.py tests/test_ddp_gpu.py -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step plain 300 python bench.py --steps 10 --warmup 3 || exit 1
for r in 1 2; do
  for s in eager window end; do
    step px_fp32_${s}_$r 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy --ddp-schedule $s || exit 1
  done
  for s in window end; do
    step px_rsag_${s}_$r 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy --reduce-dtype rsag --ddp-schedule $s || exit 1
  done
done
step plain2 300 python bench.py --steps 10 --warmup 3 || exit 1
