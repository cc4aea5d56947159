#!/bin/bash
# LayerNorm forward A/B (gamma/beta loads hoisted) via REPLICANN_SO, interleaved; LN GPU tests on the new build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
set -e
for i in 1 2 3; do
  LN_AB_FWD_ONLY=1 REPLICANN_SO=replicann_amd/ab/_C_old.so timeout -k 10 120 python scripts/ln_ab.py >> gpurun_out/r2zj_ln_old.log 2>&1
  LN_AB_FWD_ONLY=1 REPLICANN_SO=replicann_amd/ab/_C_new.so timeout -k 10 120 python scripts/ln_ab.py >> gpurun_out/r2zj_ln_new.log 2>&1
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "layer" > gpurun_out/r2zj_tests.log 2>&1
