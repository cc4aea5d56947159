#!/bin/bash
# round 4 (call O): native-vs-fp32 loss trajectories at HEAD for ViT-B/16 (its token join changed this
# round) and ResNet-18 (shortcut-gradient join), plus a GPT-2-small 2-rank self-launch rehearsal on one
# card over gloo (the bench --gpus N path).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python scripts/check_trajectory.py --model vit-b16 --steps 30 --lr 1e-4 --threshold 0.02 > gpurun_out/o_traj_vit.log 2>&1; echo "=== traj vit rc=$? $(grep -o '"max_rel_dev": [0-9.]*' gpurun_out/o_traj_vit.log)"
timeout -k 10 600 python scripts/check_trajectory.py --model resnet18 --steps 30 --threshold 0.02 > gpurun_out/o_traj_resnet.log 2>&1; echo "=== traj resnet rc=$? $(grep -o '"max_rel_dev": [0-9.]*' gpurun_out/o_traj_resnet.log)"
REPLICANN_SHARE_DEVICE=1 REPLICANN_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 4 --warmup 2 --batch 16 > gpurun_out/o_bench2.log 2>&1; echo "=== bench --gpus 2 (one card, gloo) rc=$? $(grep '^{' gpurun_out/o_bench2.log | cut -c1-300)"
exit 0
