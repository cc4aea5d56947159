#!/bin/bash
# Native RCCL communicator: GPU tests, then the GPT-2-small step as a one-rank DDP rehearsal
# (native comm graph/eager, torch ProcessGroupNCCL eager) next to the plain N=1 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
set -e
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_comm_gpu.py > gpurun_out/r2q_comm_tests.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/r2q_bench_plain.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --ddp on --comm native --graph off > gpurun_out/r2q_bench_ddp_native_eager.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --ddp on --comm torch --graph off > gpurun_out/r2q_bench_ddp_torch_eager.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --ddp on --comm native > gpurun_out/r2q_bench_ddp_native_graph.log 2>&1
