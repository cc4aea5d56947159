#!/bin/bash
# round 3: same-box A/B of the round-2 library (ab/r2_C.so) vs HEAD on the headline bench, plus
# kernel traces of the HEAD step and of the DDP step beside the comm proxy
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | tail -2 | cut -c1-400
  return $rc
}
for r in 1 2; do
  step head_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
  REPLICANN_SO=$PWD/ab/r2_C.so step r2_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
done
step lmdgrad_head 120 python scripts/gemm_one.py 65536 768 50304 nn --cfg 9 --iters 10 || exit 1
REPLICANN_SO=$PWD/ab/r2_C.so step lmdgrad_r2 120 python scripts/gemm_one.py 65536 768 50304 nn --cfg 9 --iters 10 || exit 1
step prof_head 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_head -o run -- python3 bench.py --steps 3 --warmup 2 || exit 1
REPLICANN_GEMM_RESERVE=0 step prof_proxy 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_proxy -o run -- python3 bench.py --steps 3 --warmup 2 --ddp on --comm proxy
