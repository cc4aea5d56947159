#!/bin/bash
# round 3 (session 2): full validation at HEAD — every GPU test, smoke, all BASELINE configs, perf floors
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | tail -2 | tr '\n' ' '; grep -E "passed|failed|smoke ok" gpurun_out/$n.log | tail -1
  return $rc
}
step gpu_all 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider; [ $? -ge 124 ] && exit 1
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step b_gpt2s 300 python bench.py --steps 20 --warmup 5 || exit 1
step b_gpt2m 400 python bench.py --model gpt2-medium --steps 5 --warmup 2 || exit 1
step b_gpt2m8 400 python bench.py --model gpt2-medium-fp8 --steps 5 --warmup 2 || exit 1
step b_vit 300 python bench.py --model vit-b16 --steps 10 --warmup 3 || exit 1
step b_resnet 300 python bench.py --model resnet18 --steps 20 --warmup 3 || exit 1
step b_gpt2s_2 300 python bench.py --steps 20 --warmup 5 || exit 1
