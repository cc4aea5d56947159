#!/bin/bash
# round 3 (session 2): final validation at HEAD — every GPU test, smoke, all BASELINE configs, 2-rank gloo
# rehearsal of bench.py --gpus 2 on one card, fresh GPT-2-small kernel breakdown
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"n_gpus": [0-9]*' | tail -3 | tr '\n' ' '; grep -E "passed|failed|smoke ok" gpurun_out/$n.log | tail -1
  return $rc
}
step gpu_all 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider; [ $? -ge 124 ] && exit 1
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step b_gpt2s 300 python bench.py --steps 20 --warmup 5 || exit 1
step b_gpt2m 400 python bench.py --model gpt2-medium --steps 5 --warmup 2 || exit 1
step b_gpt2m8 400 python bench.py --model gpt2-medium-fp8 --steps 5 --warmup 2 || exit 1
step b_vit 300 python bench.py --model vit-b16 --steps 10 --warmup 3 || exit 1
step b_resnet 300 python bench.py --model resnet18 --steps 20 --warmup 3 || exit 1
REPLICANN_DIST_BACKEND=gloo REPLICANN_SHARE_DEVICE=1 step gloo2 400 python bench.py --gpus 2 --steps 3 --warmup 2 || exit 1
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_zw -o run -- python3 bench.py --steps 3 --warmup 2 || exit 1
python scripts/prof_summary.py gpurun_out/prof_zw/run_kernel_trace.csv --steps 3 > gpurun_out/prof_zw_summary.txt 2>&1; head -3 gpurun_out/prof_zw_summary.txt
