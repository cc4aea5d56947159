#!/bin/bash
# round 3 (session 2): LayerNorm-backward grid (waves) after the row prefetch: A/B on ln_ab and the GPT-2 step
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | grep -o '"ms": [0-9.]*\|"ms_per_step": [0-9.]*' | tail -1
  return $rc
}
for r in 1 2; do
  for wv in 8192 4096 2048 1024; do
    REPLICANN_LN_BWD_WAVES=$wv step ln_w${wv}_$r 120 python scripts/ln_ab.py || exit 1
  done
done
for r in 1 2; do
  for wv in 8192 2048; do
    REPLICANN_LN_BWD_WAVES=$wv step g_w${wv}_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
  done
done
