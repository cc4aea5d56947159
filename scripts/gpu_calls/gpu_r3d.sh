#!/bin/bash
# round 3: leaner dynamic-queue bookkeeping — correctness, per-shape A/B (HEAD static/dynamic vs the
# round-2 library on the same box), headline bench HEAD vs r2
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | tail -3 | cut -c1-300
  return $rc
}
step sched_test 300 python -u -m pytest tests/test_gemm_sched_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
step sched_ab 300 python -u scripts/gemm_sched_ab.py --rounds 3 --reserve || exit 1
for sh in "65536 2304 768 nt" "65536 768 50304 nn" "65536 768 3072 nn" "65536 50304 768 nt"; do
  REPLICANN_SO=$PWD/ab/r2_C.so step "r2_${sh// /_}" 120 python scripts/gemm_one.py $sh --cfg 9 --iters 10 || exit 1
done
step head_1 300 python bench.py --steps 10 --warmup 3 || exit 1
REPLICANN_SO=$PWD/ab/r2_C.so step r2_1 300 python bench.py --steps 10 --warmup 3 || exit 1
