#!/bin/bash
# T6 perf regression check on the GPU: every BASELINE config's 1-GPU bench vs the committed floor.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 900 python scripts/check_perf.py --run gpt2-small gpt2-medium gpt2-medium-fp8 vit-b16 resnet18 > gpurun_out/r2zo_check_perf.log 2>&1
rc=$?
echo "exit=$rc" >> gpurun_out/r2zo_check_perf.log
exit $rc
