#!/bin/bash
# round 3 (session 2): LDS-staged stem im2col; conv tests; ResNet-18 bench
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | tail -3 | cut -c1-300
  return $rc
}
step convtest 300 python -m pytest tests/test_ops_gpu.py -q -k "im2col or conv" -p no:cacheprovider || exit 1
step im2col 120 python scripts/dev/im2col_time.py || exit 1
step bench_resnet 300 python bench.py --model resnet18 --steps 20 --warmup 3 || exit 1
step bench_resnet2 300 python bench.py --model resnet18 --steps 20 --warmup 3 || exit 1
