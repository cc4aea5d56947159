#!/bin/bash
# round 6 call O: software-pipelined 32x32 dK/dV (REPLICANN_ATTN_DKDV32 = 1 occupancy 1, 2 occupancy 2) vs the 16x16 kernel (0)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in 1 2; do for T in 256 197; do for c in 1 0; do
  echo "== DKDV32=$v T=$T causal=$c"; REPLICANN_ATTN_DKDV32=$v timeout -k 10 60 python3 scripts/dev/attn_rows.py $T $c 2>&1 | grep -v amdgpu.ids | grep "dk\|dv" || exit 1
done; done; done
O=gpurun_out/r6o.txt; : > $O
for rnd in 1 2; do for v in 0 1 2; do
  REPLICANN_ATTN_DKDV32=$v timeout -k 10 120 python3 scripts/attn_ab.py 64 --rounds 3 2>/dev/null | grep bwd | sed "s/^/dkdv32=$v /" >> $O || exit 1
  REPLICANN_ATTN_DKDV32=$v timeout -k 10 120 python3 scripts/attn_ab.py 512 --rounds 3 --T 197 --noncausal 2>/dev/null | grep bwd | sed "s/^/dkdv32=$v /" >> $O || exit 1
done; done
cat $O
