#!/bin/bash
# Re-record the GPT-2-small native-vs-fp32 100-step trajectory (lr 1e-4, b16) after the round-2 kernel changes
# (CE v2, LN-backward load hoist, dgrad epilogue alpha).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
( for i in $(seq 1 40); do date >> gpurun_out/r2zi_heartbeat.txt; sleep 20; done ) &
HB=$!
timeout -k 10 780 python scripts/check_trajectory.py --model gpt2-small --steps 100 --lr 1e-4 --threshold 0.02 --batch 16 > gpurun_out/r2zi_traj.jsonl 2> gpurun_out/r2zi_traj.err
rc=$?
kill $HB
echo "exit=$rc" >> gpurun_out/r2zi_traj.jsonl
exit $rc
