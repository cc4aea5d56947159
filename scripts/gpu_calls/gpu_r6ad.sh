#!/bin/bash
# round 6 call AD: native bf16 vs fp32 reference loss trajectories with the round-6 attention kernels (resident T <= 256 for
# ViT, 8-wave causal forward for GPT-2): same commands as round 4's call O / the GPT-2 100-step check, 30 steps
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python scripts/check_trajectory.py --model vit-b16 --steps 30 --lr 1e-4 --threshold 0.02 > gpurun_out/r6ad_traj_vit.log 2>&1; rc1=$?
echo "=== traj vit rc=$rc1 $(grep -o '"max_rel_dev": [0-9.]*' gpurun_out/r6ad_traj_vit.log)"
[ $rc1 -le 1 ] || exit $rc1
timeout -k 10 600 python scripts/check_trajectory.py --model gpt2-small --steps 30 --lr 1e-4 --threshold 0.02 > gpurun_out/r6ad_traj_gpt2.log 2>&1; rc2=$?
echo "=== traj gpt2 rc=$rc2 $(grep -o '"max_rel_dev": [0-9.]*' gpurun_out/r6ad_traj_gpt2.log)"
