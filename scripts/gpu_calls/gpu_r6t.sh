#!/bin/bash
# round 6 call T: resident backward without loop-invariant spills (opaque LDS addresses, no cs MFMA, LDS dQ bias
# reduction): numerics + timing + ViT bench
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "attention or attn" > gpurun_out/r6t_tests.log 2>&1; rc=$?
grep -E "FAIL|passed|failed" gpurun_out/r6t_tests.log | tail -12; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 scripts/attn_ab.py 512 --T 197 --noncausal --rounds 5 > gpurun_out/r6t_ab.log 2>&1 || exit 1
cut -c1-300 gpurun_out/r6t_ab.log
timeout -k 10 300 python -u bench.py --model vit-b16 --steps 10 --warmup 3 > gpurun_out/r6t_vit.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r6t_vit.log; exit 1; }
echo "vit: $(grep -o '"value": [0-9.]*' gpurun_out/r6t_vit.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6t_vit.log)"
