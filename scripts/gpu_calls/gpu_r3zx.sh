#!/bin/bash
# round 3 (session 2): LayerNorm backward with non-temporal loads of the saved forward input (REPLICANN_LN_BWD_NT, A/B)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | grep -o '"ms_per_step": [0-9.]*' | tail -1; grep -E "passed|failed" gpurun_out/$n.log | tail -1
  return $rc
}
REPLICANN_LN_BWD_NT=1 step t_ln 300 python -u -m pytest tests/test_ops_gpu.py -q -k "layer_norm or layernorm" --timeout 120 --timeout-method thread -p no:cacheprovider -x || exit 1
for r in 1 2 3; do
  step g_off_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
  REPLICANN_LN_BWD_NT=1 step g_on_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
done
