#!/bin/bash
# round 6 call Y: resident backward with the dV bias partials on the MFMA: bias-grad tests + ViT bench
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "attention or attn" > gpurun_out/r6y_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r6y_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --model vit-b16 --steps 10 --warmup 3 > gpurun_out/r6y_vit.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r6y_vit.log; exit 1; }
echo "vit: $(grep -o '"value": [0-9.]*' gpurun_out/r6y_vit.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6y_vit.log)"
