#!/bin/bash
# round 3: static/dynamic as separate instantiations — correctness, per-shape A/B, headline bench
# HEAD vs round-2 library (same box), DDP step beside the comm proxy (dynamic vs static)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | tail -2 | cut -c1-250
  return $rc
}
step sched_test 300 python -u -m pytest tests/test_gemm_sched_gpu.py "tests/test_comm_gpu.py::test_proxy_comm_keeps_data_and_orders_streams" "tests/test_comm_gpu.py::test_ddp_step_proxy_matches_native_and_enables_queue" -x -q --timeout 120 --timeout-method thread || exit 1
step sched_ab 300 python -u scripts/gemm_sched_ab.py --rounds 3 --reserve || exit 1
for r in 1 2; do
  step head_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
  REPLICANN_SO=$PWD/ab/r2_C.so step r2_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
done
step proxy_dyn 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy || exit 1
REPLICANN_GEMM_SCHED=static step proxy_static 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy || exit 1
step prof_proxy_dyn 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_proxy_dyn -o run -- python3 bench.py --steps 3 --warmup 2 --ddp on --comm proxy
