#!/bin/bash
# round 3 (session 2): fp8 resume fix + CE row kernel on raw v_exp_f32; gpu tests, smoke, bench, rocprof
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | tail -2 | cut -c1-300
  return $rc
}
step xent_ab 200 python scripts/xent_ab.py || exit 1
step gpu_all 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider; [ $? -ge 124 ] && exit 1
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench 300 python bench.py --steps 10 --warmup 3 || exit 1
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --warmup 2
