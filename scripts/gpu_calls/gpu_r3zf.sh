#!/bin/bash
# round 3 (session 2): window-schedule GPU tests + window budget sweep under the comm proxy
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | grep -o '"ms_per_step": [0-9.]*' | tail -1; grep -E "passed|failed" gpurun_out/$n.log | tail -1
  return $rc
}
step commtest 600 python -u -m pytest tests/test_comm_gpu.py -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step plain 300 python bench.py --steps 10 --warmup 3 || exit 1
for r in 1 2; do
  step px_fp32_eager_$r 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy || exit 1
  for mb in 24 40 64; do
    REPLICANN_DDP_WINDOW_MB=$mb step px_fp32_w${mb}_$r 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy --ddp-schedule window || exit 1
    REPLICANN_DDP_WINDOW_MB=$mb step px_rsag_w${mb}_$r 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy --reduce-dtype rsag --ddp-schedule window || exit 1
  done
done
