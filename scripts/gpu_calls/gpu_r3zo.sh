#!/bin/bash
# round 3 (session 2): grid caps of the LayerNorm forward and the fused optimizer (A/B on the GPT-2-small step)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | grep -o '"ms": [0-9.]*\|"ms_per_step": [0-9.]*' | tail -1
  return $rc
}
for r in 1 2; do
  for b in 2048 1024 512; do
    REPLICANN_LN_FWD_BLOCKS=$b LN_AB_FWD_ONLY=1 step lnf_b${b}_$r 120 python scripts/ln_ab.py || exit 1
  done
done
for r in 1 2; do
  step g_base_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
  REPLICANN_OPT_BLOCKS=1024 step g_opt1024_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
  REPLICANN_OPT_BLOCKS=2048 step g_opt2048_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
  REPLICANN_LN_FWD_BLOCKS=1024 step g_lnf1024_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
done
