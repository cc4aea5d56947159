#!/bin/bash
# round 3 (session 2): size threshold of the non-temporal GEMM output stores (REPLICANN_GEMM_ST_NT_MB, A/B on the step)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | grep -o '"ms_per_step": [0-9.]*' | tail -1
  return $rc
}
for r in 1 2; do
  step g_256_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
  REPLICANN_GEMM_ST_NT_MB=1024 step g_1024_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
  REPLICANN_GEMM_ST_NT_MB=350 step g_350_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
  REPLICANN_GEMM_ST_NT_MB=64 step g_64_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
done
