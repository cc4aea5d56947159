#!/bin/bash
# round 6 call AJ: resident forward waits per K/V tile (Q first, tiles in order, vmcnt(2·later tiles) + barrier) vs HEAD's
# single wait for all tiles (ab/_C_h.so), alternating on one box; numerics first
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "attention or attn" > gpurun_out/r6aj_tests.log 2>&1; rc=$?
tail -1 gpurun_out/r6aj_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|^E " gpurun_out/r6aj_tests.log | head -5; exit 1; }
for i in 1 2 3; do
REPLICANN_SO=$PWD/ab/_C_h.so timeout -k 10 200 python3 scripts/attn_ab.py 512 --T 197 --noncausal --rounds 4 > gpurun_out/r6aj_h$i.log 2>&1 || exit 1
timeout -k 10 200 python3 scripts/attn_ab.py 512 --T 197 --noncausal --rounds 4 > gpurun_out/r6aj_n$i.log 2>&1 || exit 1
echo "h$i $(grep attn_fwd gpurun_out/r6aj_h$i.log | grep -o '"ms": [0-9.]*')  n$i $(grep attn_fwd gpurun_out/r6aj_n$i.log | grep -o '"ms": [0-9.]*')"
done
