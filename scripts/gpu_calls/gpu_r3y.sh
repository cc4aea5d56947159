#!/bin/bash
# round 3 (session 2): ResNet-18 step profile (kernel trace) + the other BASELINE configs at HEAD
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | tail -2 | cut -c1-400
  return $rc
}
step bench_resnet 300 python bench.py --model resnet18 --steps 20 --warmup 3 || exit 1
step prof_resnet 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_rn -o run -- python3 bench.py --model resnet18 --steps 4 --warmup 2 || exit 1
step bench_vit 300 python bench.py --model vit-b16 --steps 10 --warmup 3 || exit 1
step bench_med 400 python bench.py --model gpt2-medium --steps 5 --warmup 2 || exit 1
step bench_med8 400 python bench.py --model gpt2-medium-fp8 --steps 5 --warmup 2 || exit 1
step bench_small 300 python bench.py --steps 10 --warmup 3 || exit 1
