#!/bin/bash
# round 3 (session 2): BatchNorm kernels — batched partial sums, hoisted per-channel constants + paired loads in the
# apply passes (A/B vs ab/ab_conv_old.so on the ResNet-18 bench); BN/conv GPU tests
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | grep -o '"value": [0-9.]*, "unit": "[a-z/]*", "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' | tail -1; grep -E "passed|failed" gpurun_out/$n.log | tail -1
  return $rc
}
step bntest 600 python -m pytest tests -q -m gpu -k "bn or batch_norm or conv or resnet or im2col or pool" -p no:cacheprovider || exit 1
for r in 1 2; do
  step rn_new_$r 300 python bench.py --model resnet18 --steps 20 --warmup 3 || exit 1
  REPLICANN_SO=$PWD/ab/ab_conv_old.so step rn_old_$r 300 python bench.py --model resnet18 --steps 20 --warmup 3 || exit 1
done
step prof_rn 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_rn2 -o run -- python3 bench.py --model resnet18 --steps 4 --warmup 2 || exit 1
