#!/bin/bash
# round 3: dynamic GEMM tile queue — correctness (bitwise vs static), proxy comm, interleaved A/B
# timing, headline bench static vs dynamic, and the DDP step beside the comm proxy
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | tail -4
  return $rc
}
true
step sched_ab 300 python -u scripts/gemm_sched_ab.py --rounds 5 --reserve 8 16 || exit 1
step bench_dyn 300 python bench.py --steps 10 --warmup 3 || exit 1
REPLICANN_GEMM_SCHED=static step bench_static 300 python bench.py --steps 10 --warmup 3 || exit 1
REPLICANN_GEMM_SCHED=static REPLICANN_GEMM_RESERVE=0 step proxy_static_r0 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy || exit 1
REPLICANN_GEMM_RESERVE=0 step proxy_dyn_r0 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy || exit 1
REPLICANN_GEMM_RESERVE=8 step proxy_dyn_r8 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy || exit 1
REPLICANN_GEMM_RESERVE=16 step proxy_dyn_r16 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy || exit 1
REPLICANN_GEMM_SCHED=static REPLICANN_GEMM_RESERVE=8 step proxy_static_r8 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy
