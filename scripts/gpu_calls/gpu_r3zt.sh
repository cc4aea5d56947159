#!/bin/bash
# round 3 (session 2): non-temporal loads / stores in the CE row kernel (REPLICANN_XENT_NT 0..3, A/B)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | grep -o '"ms_per_step": [0-9.]*\|"v2_ms": [0-9.]*' | tail -1; grep -E "passed|failed" gpurun_out/$n.log | tail -1
  return $rc
}
REPLICANN_XENT_NT=3 step t_xent 300 python -u -m pytest tests/test_ops_gpu.py -q -k "cross_entropy or xent" --timeout 120 --timeout-method thread -p no:cacheprovider -x || exit 1
for r in 1 2; do
  for k in 0 1 2 3; do
    REPLICANN_XENT_NT=$k step xent_nt${k}_$r 200 python scripts/xent_ab.py || exit 1
  done
done
for r in 1 2; do
  step g_nt0_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
  REPLICANN_XENT_NT=3 step g_nt3_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
  REPLICANN_XENT_NT=2 step g_nt2_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
done
