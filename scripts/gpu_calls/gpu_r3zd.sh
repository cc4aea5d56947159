#!/bin/bash
# round 3 (session 2): DDP rsag reducer (fp32 reduce-scatter + bf16 all-gather) — GPU tests, and the
# GPT-2-small step under the 8-GPU comm proxy: fp32 all-reduce vs rsag vs bf16 all-reduce
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | tail -2 | cut -c1-260
  return $rc
}
step commtest 600 python -u -m pytest tests/test_comm_gpu.py tests/test_ddp_gpu.py -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step plain 300 python bench.py --steps 10 --warmup 3 || exit 1
for r in 1 2; do
  for m in fp32 rsag bf16; do
    step px_${m}_$r 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy --reduce-dtype $m || exit 1
  done
done
step plain2 300 python bench.py --steps 10 --warmup 3 || exit 1
