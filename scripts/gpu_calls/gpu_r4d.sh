#!/bin/bash
# round 4 (call D): causal D=64 attention kernel variants — fp32-reference tests of the 64-queries-per-
# wave forward and the 4-group dQ / dK-dV backward, then GPT-2-small-shape timings of every arm.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
PT="python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $PT tests/test_ops_gpu.py -k "attention" > gpurun_out/attn_tests.log 2>&1; rc=$?
echo "=== attn_tests rc=$rc"; grep -E "passed|failed" gpurun_out/attn_tests.log | tail -1
grep -E "^E  |FAILED" gpurun_out/attn_tests.log | head -20
if grep -q "illegal memory access\|hipErrorIllegalAddress\|HSA_STATUS_ERROR\|Memory access fault" gpurun_out/attn_tests.log; then
  echo "GPU FAULT"; exit 2
fi
[ $rc -ne 0 ] && exit 1
for r in 1 2; do
  for arm in "2 2 2" "4 2 2" "2 4 2" "2 2 4" "4 4 4"; do
    set -- $arm
    REPLICANN_ATTN_FWD_QI=$1 REPLICANN_ATTN_DQ_QG=$2 REPLICANN_ATTN_DKDV_KG=$3 \
      timeout -k 10 120 python scripts/attn_ab.py 64 --rounds 3 > gpurun_out/attn_ab_$1$2$3_$r.log 2>&1 || { echo "attn_ab $arm failed"; exit 1; }
    echo "arm qi=$1 qg=$2 kg=$3 r$r: $(grep -o '"op": "[a-z_]*".*"tflops": [0-9.]*' gpurun_out/attn_ab_$1$2$3_$r.log | sed 's/, "B".*"ms"/ ms/' | tr '\n' ' ')"
  done
done
exit 0
