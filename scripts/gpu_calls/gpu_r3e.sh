#!/bin/bash
# round 3: (a) per-kernel step profiles of HEAD vs the round-2 library on one box;
# (b) persistent-GEMM epilogue ablations (dev library ab/dev_C.so: cfg 90 + DBG; outputs wrong)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | grep "^{" | tail -3 | cut -c1-200
  return $rc
}
step prof_head 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_head -o run -- python3 bench.py --steps 3 --warmup 2 || exit 1
REPLICANN_SO=$PWD/ab/r2_C.so step prof_r2 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r2 -o run -- python3 bench.py --steps 3 --warmup 2 || exit 1
for sh in "65536 2304 768 nt" "65536 768 3072 nt" "65536 768 50304 nn"; do
  for r in 1 2; do
    for cfg in 9 94 122 154 91 106; do
      REPLICANN_SO=$PWD/ab/dev_C.so REPLICANN_DEV=1 REPLICANN_GEMM_SCHED=static step "abl_${sh// /_}_c${cfg}_r$r" 120 python scripts/gemm_one.py $sh --cfg $cfg --iters 10 || exit 1
    done
  done
done
