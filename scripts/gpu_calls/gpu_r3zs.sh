#!/bin/bash
# round 3 (session 2): one-pass column sums up to 1024 partial rows (A/B vs the two-stage kernel, GPT-2 and ResNet)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | grep -o '"ms_per_step": [0-9.]*' | tail -1; grep -E "passed|failed" gpurun_out/$n.log | tail -1
  return $rc
}
step t_ops 300 python -u -m pytest tests/test_ops_gpu.py tests/test_determinism_gpu.py -q --timeout 120 --timeout-method thread -p no:cacheprovider -x || exit 1
for r in 1 2; do
  step g_new_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
  REPLICANN_COLSUM_1PASS=0 step g_old_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
  step r_new_$r 300 python bench.py --model resnet18 --steps 20 --warmup 3 || exit 1
  REPLICANN_COLSUM_1PASS=0 step r_old_$r 300 python bench.py --model resnet18 --steps 20 --warmup 3 || exit 1
done
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_zs -o run -- python3 bench.py --steps 3 --warmup 2 || exit 1
python scripts/prof_summary.py gpurun_out/prof_zs/run_kernel_trace.csv --steps 3 > gpurun_out/prof_zs_summary.txt 2>&1; grep -i "colsum\|kernel-busy" gpurun_out/prof_zs_summary.txt
step rprof_new 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_zs_rn -o run -- python3 bench.py --model resnet18 --steps 3 --warmup 2 || exit 1
python scripts/prof_summary.py gpurun_out/prof_zs_rn/run_kernel_trace.csv --steps 3 > gpurun_out/prof_zs_rn_summary.txt 2>&1; grep -i "colsum\|colred\|kernel-busy" gpurun_out/prof_zs_rn_summary.txt
