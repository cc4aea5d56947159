#!/bin/bash
# round 3: DDP bucket size under the comm proxy (overlap vs one late collective)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | tail -1 | cut -c1-200
  return $rc
}
step plain 300 python bench.py --steps 10 --warmup 3 || exit 1
for b in 64 1000 16 256 64; do
  step px_b$b 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy --bucket-mb $b || exit 1
done
