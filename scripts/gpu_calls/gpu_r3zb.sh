#!/bin/bash
# round 3 (session 2): attention forward skips invisible 16-key column blocks in masked tiles and dead
# query waves (A/B vs ab/ab_attn_old.so at GPT-2 causal T=1024 and ViT T=197); attention tests
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | tail -3 | cut -c1-250
  return $rc
}
step attn_t 300 python -m pytest tests -q -m gpu -k "attn or attention or reference_parity or determinism" -p no:cacheprovider || exit 1
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export REPLICANN_SO=$PWD/ab/ab_attn_old.so; else unset REPLICANN_SO; fi
    step g_${v}_$r 200 python scripts/attn_ab.py 64 --fwd 3 --bwd 2 --rounds 4 || exit 1
    step v_${v}_$r 200 python scripts/attn_ab.py 512 --T 197 --noncausal --fwd 3 --bwd 2 --rounds 4 || exit 1
  done
done
