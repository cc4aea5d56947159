#!/bin/bash
# round 3 (session 2): split-K reduction with 4 slab loads in flight per thread (REPLICANN_SPLITK_BATCH, A/B)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | grep -o '"ms_per_step": [0-9.]*' | tail -1; grep -E "passed|failed|smoke ok" gpurun_out/$n.log | tail -1
  return $rc
}
step gpu_all 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
for r in 1 2 3; do
  step g_new_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
  REPLICANN_SPLITK_BATCH=0 step g_old_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
done
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_zz -o run -- python3 bench.py --steps 3 --warmup 2 || exit 1
python scripts/prof_summary.py gpurun_out/prof_zz/run_kernel_trace.csv --steps 3 > gpurun_out/prof_zz_summary.txt 2>&1; grep -i "splitk\|kernel-busy" gpurun_out/prof_zz_summary.txt
