#!/bin/bash
# Checkpoint: full GPU suite + smoke() + headline bench + one-rank RCCL DDP rehearsal.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
set -e
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r2za_gpu_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2za_smoke.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2za_bench.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --ddp on > gpurun_out/r2za_bench_ddp.log 2>&1
