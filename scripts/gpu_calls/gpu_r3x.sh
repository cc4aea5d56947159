#!/bin/bash
# round 3 (session 2): attention forward variant 4 (deferred max, guide T13) vs 3; numerics via the attention tests
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | tail -4 | cut -c1-300
  return $rc
}
REPLICANN_ATTN_FWD=4 step attn_t4 300 python -m pytest tests -q -m gpu -k "attn or attention or reference_parity or convergence" -p no:cacheprovider
step ab 300 python scripts/attn_ab.py 64 --fwd 3,4 --bwd 2 --rounds 4 || exit 1
step abnc 300 python scripts/attn_ab.py 64 --fwd 3,4 --bwd 2 --rounds 3 --noncausal || exit 1
