#!/bin/bash
# The driver's multi-GPU bench command shape, rehearsed on one card: torchrun N=2, both ranks on
# cuda:0, collectives over gloo (RCCL refuses two ranks on one device).  Checks bench.py's
# multi-rank path end to end (rendezvous, DDP, pre-step tuning pass, barrier + max-over-ranks timing, JSON).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
set -e
export REPLICANN_DIST_BACKEND=gloo REPLICANN_SHARE_DEVICE=1
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --batch 16 > gpurun_out/r2u_torchrun2_gloo.log 2>&1
