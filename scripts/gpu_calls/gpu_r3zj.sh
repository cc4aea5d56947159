#!/bin/bash
# round 3 (session 2): conv wgrad split-K target (REPLICANN_CONVW_TARGET workgroups) A/B on the ResNet-18 bench
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | grep -o '"ms_per_step": [0-9.]*' | tail -1
  return $rc
}
for r in 1 2; do
  for t in 512 256 384 768; do
    REPLICANN_CONVW_TARGET=$t step rn_t${t}_$r 300 python bench.py --model resnet18 --steps 20 --warmup 3 || exit 1
  done
done
