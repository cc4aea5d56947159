#!/bin/bash
# round 6 call U: resident backward scheduling A/B: (h) committed (ab/_C_h.so), (a) P2 S/dP chains before the softmax VALU (ab/_C_a.so) vs
# (b) + P1 transposed fragments read ahead of the VALU (tree _C.so); numerics of (b)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "attention_resident or attention_d64 or bias_grad" > gpurun_out/r6u_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r6u_tests.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
REPLICANN_SO=$PWD/ab/_C_h.so timeout -k 10 200 python3 scripts/attn_ab.py 512 --T 197 --noncausal --rounds 5 > gpurun_out/r6u_h$i.log 2>&1 || exit 1
echo "h$i: $(grep attn_bwd gpurun_out/r6u_h$i.log | cut -c1-120)"
REPLICANN_SO=$PWD/ab/_C_a.so timeout -k 10 200 python3 scripts/attn_ab.py 512 --T 197 --noncausal --rounds 5 > gpurun_out/r6u_a$i.log 2>&1 || exit 1
timeout -k 10 200 python3 scripts/attn_ab.py 512 --T 197 --noncausal --rounds 5 > gpurun_out/r6u_b$i.log 2>&1 || exit 1
echo "a$i: $(grep attn_bwd gpurun_out/r6u_a$i.log | cut -c1-120)"; echo "b$i: $(grep attn_bwd gpurun_out/r6u_b$i.log | cut -c1-120)"
done
