#!/bin/bash
# round 3 (session 2): short-key attention forward with all K/V staged up front (variant 3 at Tk <= 256)
# vs the streaming kernel (variant 5 = same kernel family, per-tile hand-off); attention tests
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | grep attn_fwd | tail -3 | cut -c1-250; grep -E "passed|failed" gpurun_out/$n.log | tail -1
  return $rc
}
step attn_t 300 python -m pytest tests -q -m gpu -k "attn or attention or reference_parity or determinism or vit" -p no:cacheprovider || exit 1
step v 200 python scripts/attn_ab.py 512 --T 197 --noncausal --fwd 3,5 --bwd 2 --rounds 5 || exit 1
step vc 200 python scripts/attn_ab.py 512 --T 197 --fwd 3,5 --bwd 2 --rounds 4 || exit 1
