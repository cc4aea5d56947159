#!/bin/bash
# round 3 (session 2): rsag for the tied wte (per-contribution fp32 reduce-scatters, one bf16 all-gather of the
# summed shards); GPU DDP/comm tests; proxy step vs plain
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | grep -o '"ms_per_step": [0-9.]*' | tail -1; grep -E "passed|failed" gpurun_out/$n.log | tail -1
  return $rc
}
step commtest 900 python -u -m pytest tests/test_comm_gpu.py tests/test_ddp_gpu.py tests/test_convergence_gpu.py -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
for r in 1 2; do
  step plain_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
  step px_default_$r 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy || exit 1
  step px_fp32_eager_$r 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy --reduce-dtype fp32 --ddp-schedule eager || exit 1
done
