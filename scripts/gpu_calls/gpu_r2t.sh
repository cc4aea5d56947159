#!/bin/bash
# Checkpoint: full GPU test suite (incl. native comm, pre-step tuning pass, xent v2, fp8 kernels) + smoke().
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
set -e
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r2t_gpu_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2t_smoke.log 2>&1
