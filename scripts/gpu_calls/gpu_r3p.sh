#!/bin/bash
# round 3: LayerNorm-backward grid size (partial rows for the column reductions) A/B on the headline step;
# 2-rank self-launched bench on one card over gloo (flow check of --gpus 2, not a perf number)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | tail -1 | cut -c1-260
  return $rc
}
for w in 8192 2048 4096 8192 2048; do
  REPLICANN_LN_BWD_WAVES=$w step ln_$w 300 python bench.py --steps 10 --warmup 3 || exit 1
done
REPLICANN_DIST_BACKEND=gloo REPLICANN_SHARE_DEVICE=1 step gpus2_gloo 400 python bench.py --gpus 2 --steps 3 --warmup 2 || exit 1
