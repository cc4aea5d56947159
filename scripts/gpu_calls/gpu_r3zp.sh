#!/bin/bash
# round 3 (session 2): non-temporal stores for the saved gelu'(h) of the fc1 forward epilogue (A/B)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | grep -o '"ms": [0-9.]*\|"ms_per_step": [0-9.]*\|[0-9.]* ms' | tail -1
  return $rc
}
for r in 1 2; do
  step fc1_base_$r 120 python scripts/gemm_one.py 65536 3072 768 nt --act 5 --bias --cfg 9 || exit 1
  REPLICANN_GEMM_PRE_NT=1 step fc1_prent_$r 120 python scripts/gemm_one.py 65536 3072 768 nt --act 5 --bias --cfg 9 || exit 1
done
for r in 1 2; do
  step g_base_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
  REPLICANN_GEMM_PRE_NT=1 step g_prent_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
done
