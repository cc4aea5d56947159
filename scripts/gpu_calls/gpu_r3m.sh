#!/bin/bash
# round 3: ResNet-18 step breakdown (graph replay traced, split at the SGD kernel) + GPT-2-medium bf16 vs fp8
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | tail -2 | cut -c1-300
  return $rc
}
step rn18 300 python bench.py --model resnet18 --steps 20 --warmup 3 || exit 1
step prof_rn18 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_rn18 -o run -- python3 bench.py --model resnet18 --steps 5 --warmup 3 || exit 1
step g2m 400 python bench.py --model gpt2-medium --steps 5 --warmup 3 || exit 1
step g2m_fp8 400 python bench.py --model gpt2-medium-fp8 --steps 5 --warmup 3 || exit 1
