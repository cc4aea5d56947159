#!/bin/bash
# Native comm with recordStream lifetimes: comm GPU tests + one-rank DDP bench (native, graph and eager).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
set -e
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_comm_gpu.py > gpurun_out/r2ze_comm_tests.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --ddp on > gpurun_out/r2ze_bench_ddp_graph.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --ddp on --graph off > gpurun_out/r2ze_bench_ddp_eager.log 2>&1
timeout -k 10 200 python scripts/comm_bench.py 1,64 > gpurun_out/r2ze_comm_bench.log 2>&1
