#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r2p
set -e
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2p -o g2s -- python bench.py --steps 5 --warmup 3 --graph off > gpurun_out/prof_r2p.log 2>&1
