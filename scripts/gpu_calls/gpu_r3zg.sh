#!/bin/bash
# round 3 (session 2): new DDP defaults (rsag reducer + auto window schedule): full GPU tests, smoke,
# 2-rank-on-one-card gloo rehearsal of bench.py --gpus 2, proxy step, plain bench
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | grep -o '"ms_per_step": [0-9.]*\|"n_gpus": [0-9]*' | tail -2 | tr '\n' ' '; grep -E "passed|failed|smoke ok" gpurun_out/$n.log | tail -1
  return $rc
}
step gpu_all 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider; [ $? -ge 124 ] && exit 1
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench 300 python bench.py --steps 10 --warmup 3 || exit 1
REPLICANN_DIST_BACKEND=gloo REPLICANN_SHARE_DEVICE=1 step gloo2 400 python bench.py --gpus 2 --steps 3 --warmup 2 || exit 1
step px_default 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy || exit 1
step px_fp32_eager 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy --reduce-dtype fp32 --ddp-schedule eager || exit 1
step px_default2 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy || exit 1
