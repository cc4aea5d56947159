#!/bin/bash
# torchrun N=2 bench rehearsal on one card (gloo) with the rank-0 tuning-table broadcast; then the comm/DDP GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
set -e
REPLICANN_DIST_BACKEND=gloo REPLICANN_SHARE_DEVICE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --batch 16 > gpurun_out/r2zf_torchrun2.log 2>&1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_comm_gpu.py tests/test_ddp_gpu.py > gpurun_out/r2zf_tests.log 2>&1
