#!/bin/bash
# round 3 (session 2): GELU epilogue A/B (old helpers in ab/ab_gelu_old.so vs tree), optimizer-load fix check
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | tail -3 | cut -c1-300
  return $rc
}
step fp8dbg 200 python scripts/dev/fp8_resume_debug.py
step fp8t 200 python -m pytest tests/test_fp8_state.py -q -m gpu -p no:cacheprovider
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export REPLICANN_SO=$PWD/ab/ab_gelu_old.so; else unset REPLICANN_SO; fi
    step g5_${v}_$r 120 python scripts/gemm_one.py 65536 3072 768 nt --act 5 --bias --cfg 9 --iters 100 || exit 1
    step g6_${v}_$r 120 python scripts/gemm_one.py 65536 3072 768 nn --act 6 --cfg 9 --iters 100 || exit 1
  done
done
unset REPLICANN_SO
step bench_new 300 python bench.py --steps 10 --warmup 3 || exit 1
REPLICANN_SO=$PWD/ab/ab_gelu_old.so step bench_old 300 python bench.py --steps 10 --warmup 3 || exit 1
step bench_new2 300 python bench.py --steps 10 --warmup 3 || exit 1
