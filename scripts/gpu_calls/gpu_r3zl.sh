#!/bin/bash
# round 3 (session 2): row-mapped max-pool backward; pool/conv tests; ResNet-18 bench + profile
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | tail -2 | tr '\n' ' '; grep -E "passed|failed" gpurun_out/$n.log | tail -1
  return $rc
}
step tests 600 python -m pytest tests/test_ops_gpu.py tests/test_convergence_gpu.py -q -k "pool or conv or resnet" -p no:cacheprovider || exit 1
step rn_1 300 python bench.py --model resnet18 --steps 20 --warmup 3 || exit 1
step rn_2 300 python bench.py --model resnet18 --steps 20 --warmup 3 || exit 1
step prof_rn 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_rn4 -o run -- python3 bench.py --model resnet18 --steps 4 --warmup 2 || exit 1
