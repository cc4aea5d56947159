#!/bin/bash
# Final round-2 GPT-2-small b64 per-step kernel breakdown (eager) after CE v2 / LN-bwd changes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r2zb
set -e
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_r2zb/g2s -o g2s -- python bench.py --steps 5 --warmup 3 --graph off > gpurun_out/prof_r2zb/g2s.log 2>&1
python scripts/prof_steps.py "$(find gpurun_out/prof_r2zb/g2s -name '*.db' | head -n1)" --steps 5 --per-step 12 --top 32 > gpurun_out/prof_r2zb/g2s_steps.txt
find gpurun_out/prof_r2zb -name "*.db" -delete
