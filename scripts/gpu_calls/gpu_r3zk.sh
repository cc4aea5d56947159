#!/bin/bash
# round 3 (session 2): grouped pre-reduction of tall split-K slab stacks (conv weight gradients, stem wgrad);
# GEMM/conv GPU tests; ResNet-18 A/B vs ab/ab_splitk_old.so + profile
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | tail -2 | tr '\n' ' '; grep -E "passed|failed" gpurun_out/$n.log | tail -1
  return $rc
}
step tests 900 python -m pytest tests/test_ops_gpu.py tests/test_convergence_gpu.py -q -k "gemm or split or conv or bn or resnet or im2col" -p no:cacheprovider || exit 1
for r in 1 2; do
  step rn_new_$r 300 python bench.py --model resnet18 --steps 20 --warmup 3 || exit 1
  REPLICANN_SO=$PWD/ab/ab_splitk_old.so step rn_old_$r 300 python bench.py --model resnet18 --steps 20 --warmup 3 || exit 1
done
step prof_rn 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_rn3 -o run -- python3 bench.py --model resnet18 --steps 4 --warmup 2 || exit 1
