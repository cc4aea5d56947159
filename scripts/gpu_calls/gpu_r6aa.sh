#!/bin/bash
# round 6 call AA: resident backward with δ from registers (one barrier less per head) and per-phase fragment offsets;
# numerics, then alternating on one box vs HEAD (ab/_C_h.so): attention timing and the ViT-B/16 step
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "attention or attn" > gpurun_out/r6aa_tests.log 2>&1; rc=$?
tail -1 gpurun_out/r6aa_tests.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
REPLICANN_SO=$PWD/ab/_C_h.so timeout -k 10 200 python3 scripts/attn_ab.py 512 --T 197 --noncausal --rounds 4 > gpurun_out/r6aa_ah$i.log 2>&1 || exit 1
timeout -k 10 200 python3 scripts/attn_ab.py 512 --T 197 --noncausal --rounds 4 > gpurun_out/r6aa_an$i.log 2>&1 || exit 1
echo "h$i $(grep attn_bwd gpurun_out/r6aa_ah$i.log | grep -o '"ms": [0-9.]*')  n$i $(grep attn_bwd gpurun_out/r6aa_an$i.log | grep -o '"ms": [0-9.]*')"
done
for i in 1 2; do
REPLICANN_SO=$PWD/ab/_C_h.so timeout -k 10 300 python -u bench.py --model vit-b16 --steps 10 --warmup 3 > gpurun_out/r6aa_h$i.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --model vit-b16 --steps 10 --warmup 3 > gpurun_out/r6aa_n$i.log 2>&1 || exit 1
echo "vit h$i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6aa_h$i.log)  n$i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6aa_n$i.log)"
done
