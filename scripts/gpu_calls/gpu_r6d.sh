#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for T in 256 197; do for c in 1 0; do
  echo "== ATTN32=1 T=$T causal=$c"; REPLICANN_ATTN32=1 timeout -k 10 60 python3 scripts/dev/attn_rows.py $T $c 2>&1 | grep -v amdgpu.ids || exit 1
done; done
