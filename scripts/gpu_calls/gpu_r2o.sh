#!/bin/bash
# Round-2 final validation: full GPU test suite, smoke(), N=1 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
set -e
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/final_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/final_bench.log 2>&1
