#!/bin/bash
# Round-2 GPU call: GELU saved-derivative epilogues — tests + bench A/B (REPLICANN_MLP_GELU=pre = old path).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ops_gpu.py tests/test_models.py tests/test_convergence_gpu.py > gpurun_out/gelu_tests.log 2>&1
for v in pre deriv pre deriv; do
  REPLICANN_MLP_GELU=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b_$v.log 2>&1
  echo "$v $(tail -1 gpurun_out/b_$v.log | cut -c1-200)" >> gpurun_out/gelu_ab.log
done
