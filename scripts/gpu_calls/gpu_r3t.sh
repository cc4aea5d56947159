#!/bin/bash
# round 3 (session 2): fp8 resume debug; GELU epilogue constants folded (fc1 fwd GELU_D / fc2 dgrad MUL_BWD timing); bench
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | tail -12 | cut -c1-300
  return $rc
}
step fp8dbg 200 python scripts/dev/fp8_resume_debug.py
step g5 120 python scripts/gemm_one.py 65536 3072 768 nt --act 5 --bias --cfg 9 || exit 1
step g6 120 python scripts/gemm_one.py 65536 3072 768 nn --act 6 --cfg 9 || exit 1
step g0 120 python scripts/gemm_one.py 65536 3072 768 nt --bias --cfg 9 || exit 1
step g0n 120 python scripts/gemm_one.py 65536 3072 768 nn --cfg 9 || exit 1
step bench 300 python bench.py --steps 10 --warmup 3 || exit 1
