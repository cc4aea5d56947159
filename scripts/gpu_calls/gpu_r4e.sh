#!/bin/bash
# HISTORICAL (kept as the record of round-4 call E): the REPLICANN_ATTN_DQ_QG / REPLICANN_ATTN_DKDV_KG
# knobs it sets were removed in commit b263165, so on the current library every arm runs the default
# kernel and the A/B would compare nothing.  It refuses to run.
echo "gpu_r4e.sh is historical: its attention knobs no longer exist (b263165)" >&2; exit 2
# round 4 (call E): software-pipelined D=64 attention forward (REPLICANN_ATTN_FWD_PIPE 1 / 2) —
# fp32-reference tests of every attention arm, forward A/B at GPT-2-small shapes, per-kernel times
# of the backward arms (kernel trace), attention PMC of the default arm.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
PT="python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $PT tests/test_ops_gpu.py -k "attention" > gpurun_out/attn_tests_e.log 2>&1; rc=$?
echo "=== attn_tests rc=$rc"; grep -E "passed|failed" gpurun_out/attn_tests_e.log | tail -1
grep -E "^E  |FAILED" gpurun_out/attn_tests_e.log | head -20
if grep -q "illegal memory access\|hipErrorIllegalAddress\|HSA_STATUS_ERROR\|Memory access fault" gpurun_out/attn_tests_e.log; then
  echo "GPU FAULT"; exit 2
fi
[ $rc -ne 0 ] && exit 1
for r in 1 2 3; do
  for pipe in 0 1 2; do
    REPLICANN_ATTN_FWD_PIPE=$pipe timeout -k 10 120 python scripts/attn_ab.py 64 --rounds 3 > gpurun_out/attn_pipe_${pipe}_$r.log 2>&1 || { echo "attn_ab pipe $pipe failed"; exit 1; }
    echo "pipe=$pipe r$r: $(grep -o '"op": "[a-z_]*".*"tflops": [0-9.]*' gpurun_out/attn_pipe_${pipe}_$r.log | sed 's/, "B".*"ms"/ ms/' | tr '\n' ' ')"
  done
done
for arm in "2 2" "4 2" "2 4" "4 4"; do
  set -- $arm
  REPLICANN_ATTN_DQ_QG=$1 REPLICANN_ATTN_DKDV_KG=$2 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/attn_kt_$1$2 -o run -- python3 scripts/attn_ab.py 64 --rounds 2 > /dev/null 2>&1 || { echo "trace $arm failed"; exit 1; }
  echo "qg=$1 kg=$2:"; python -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'attn' in r['Name']: print('  %8.1f us x%s  %s' % (float(r['AverageNs'])/1e3, r['Calls'], r['Name'][:90]))
" gpurun_out/attn_kt_$1$2/run_kernel_stats.csv
done
timeout -k 10 400 bash scripts/pmc_attn.sh "64 --rounds 1" attn4 > gpurun_out/pmc_attn.log 2>&1 || { echo "pmc failed"; exit 1; }
python scripts/pmc_summary.py gpurun_out/pmc_attn/attn4*_counter_collection.csv --match attn > gpurun_out/pmc_attn_summary.txt 2>&1
cat gpurun_out/pmc_attn_summary.txt | head -30
exit 0
