#!/bin/bash
# round 3 (session 2): act-backward GEMM epilogue loads both aux halves up front (A/B vs ab/ab_pk_old.so)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | tail -3 | cut -c1-300
  return $rc
}
step gemmtest 600 python -m pytest tests/test_ops_gpu.py -q -k "gemm or mlp or act" -p no:cacheprovider || exit 1
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export REPLICANN_SO=$PWD/ab/ab_pk_old.so; else unset REPLICANN_SO; fi
    step g6_${v}_$r 120 python scripts/gemm_one.py 65536 3072 768 nn --act 6 --cfg 9 --iters 100 || exit 1
    step g4_${v}_$r 120 python scripts/gemm_one.py 65536 3072 768 nn --act 4 --cfg 9 --iters 100 || exit 1
  done
done
unset REPLICANN_SO
step bench_new 300 python bench.py --steps 10 --warmup 3 || exit 1
REPLICANN_SO=$PWD/ab/ab_pk_old.so step bench_old 300 python bench.py --steps 10 --warmup 3 || exit 1
step bench_new2 300 python bench.py --steps 10 --warmup 3 || exit 1
