#!/bin/bash
# round 6 call AH: dQ bias partials by an in-register reduce-scatter (no LDS round trip, two barriers fewer per head):
# bias-gradient tests, then bias / plain timing alternating (r6ag: plain 0.487 / 0.499, bias 0.542 / 0.553 ms)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "attention or attn" > gpurun_out/r6ah_tests.log 2>&1; rc=$?
tail -1 gpurun_out/r6ah_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|^E " gpurun_out/r6ah_tests.log | head -5; exit 1; }
for i in 1 2; do
timeout -k 10 200 python3 scripts/attn_ab.py 512 --T 197 --noncausal --rounds 4 > gpurun_out/r6ah_n$i.log 2>&1 || exit 1
timeout -k 10 200 python3 scripts/attn_ab.py 512 --T 197 --noncausal --rounds 4 --bias-grad > gpurun_out/r6ah_b$i.log 2>&1 || exit 1
echo "plain$i $(grep attn_bwd gpurun_out/r6ah_n$i.log | grep -o '"ms": [0-9.]*')  bias$i $(grep attn_bwd gpurun_out/r6ah_b$i.log | grep -o '"ms": [0-9.]*')"
done
timeout -k 10 300 python -u bench.py --model vit-b16 --steps 10 --warmup 3 > gpurun_out/r6ah_vit.log 2>&1 || exit 1
echo "vit: $(grep -o '"value": [0-9.]*' gpurun_out/r6ah_vit.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6ah_vit.log)"
