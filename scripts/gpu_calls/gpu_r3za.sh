#!/bin/bash
# round 3 (session 2): step profiles at HEAD (GPT-2 small headline, ViT-B/16)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | tail -2 | cut -c1-300
  return $rc
}
step prof_g 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_g -o run -- python3 bench.py --steps 4 --warmup 2 || exit 1
step prof_v 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_v -o run -- python3 bench.py --model vit-b16 --steps 4 --warmup 2 || exit 1
step bench_g 300 python bench.py --steps 10 --warmup 3 || exit 1
