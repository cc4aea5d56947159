#!/bin/bash
# round 6 call W: attention accuracy (float64 reference) and the cross-decoder parity errors, pre-resident build
# (ab/_C_old.so, commit 8c2efb3) vs the tree
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
REPLICANN_SO=$PWD/ab/_C_old.so timeout -k 10 300 python3 scripts/dev/attn_err.py > gpurun_out/r6w_old.log 2>&1 || { tail -5 gpurun_out/r6w_old.log; exit 1; }
timeout -k 10 300 python3 scripts/dev/attn_err.py > gpurun_out/r6w_new.log 2>&1 || { tail -5 gpurun_out/r6w_new.log; exit 1; }
grep case gpurun_out/r6w_old.log; grep case gpurun_out/r6w_new.log
