#!/bin/bash
# round 3 (session 2): LayerNorm fwd/bwd with a one-row software prefetch (A/B vs ab/ab_ln_old.so), LN tests, bench
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | tail -3 | cut -c1-300
  return $rc
}
step lntest 300 python -m pytest tests/test_ops_gpu.py -q -k "layer_norm or layernorm or ln" -p no:cacheprovider || exit 1
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export REPLICANN_SO=$PWD/ab/ab_ln_old.so; else unset REPLICANN_SO; fi
    step ln_${v}_$r 120 python scripts/ln_ab.py || exit 1
    LN_AB_FWD_ONLY=1 step lnf_${v}_$r 120 python scripts/ln_ab.py || exit 1
  done
done
unset REPLICANN_SO
step bench_new 300 python bench.py --steps 10 --warmup 3 || exit 1
REPLICANN_SO=$PWD/ab/ab_ln_old.so step bench_old 300 python bench.py --steps 10 --warmup 3 || exit 1
step bench_new2 300 python bench.py --steps 10 --warmup 3 || exit 1
