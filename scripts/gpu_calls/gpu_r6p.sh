#!/bin/bash
# round 6 call P: the new forced-rescale attention test; the driver's multi-GPU bench command shape rehearsed on one card
# (torchrun N=2, both ranks on cuda:0, gloo); the comm / DDP GPU tests
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "fwd32_deferred or attention_d64" > gpurun_out/r6p_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|passed|failed" gpurun_out/r6p_tests.log | tail -12; [ $rc -eq 0 ] || exit 1
REPLICANN_DIST_BACKEND=gloo REPLICANN_SHARE_DEVICE=1 timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --batch 16 > gpurun_out/r6p_torchrun2.log 2>&1 || { echo "torchrun2 failed"; tail -20 gpurun_out/r6p_torchrun2.log; exit 1; }
grep metric gpurun_out/r6p_torchrun2.log | cut -c1-600
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_comm_gpu.py tests/test_ddp_gpu.py > gpurun_out/r6p_ddp_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r6p_ddp_tests.log; exit $rc
