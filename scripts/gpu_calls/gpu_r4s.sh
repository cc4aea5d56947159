#!/bin/bash
# round 4 (call S): skinny-M decode GEMM (config 10): GEMM tests, the GEMM + generation + determinism
# GPU tests, decode throughput of GPT-2-small at batch 1 / 16 / 64 and a kernel profile of batch-16 decode.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
fault() { grep -q "illegal memory access\|hipErrorIllegalAddress\|HSA_STATUS_ERROR\|Memory access fault" "$1"; }
PT="python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $PT -x tests/test_ops_gpu.py -k "skinny" > gpurun_out/s_skinny.log 2>&1; rc=$?
echo "=== s_skinny rc=$rc $(grep -E 'passed|failed' gpurun_out/s_skinny.log | tail -1)"; grep -E "FAILED|Error" gpurun_out/s_skinny.log | head
fault gpurun_out/s_skinny.log && exit 2; [ $rc -ne 0 ] && exit 1
timeout -k 10 600 $PT tests/test_ops_gpu.py tests/test_generate_gpu.py tests/test_determinism_gpu.py > gpurun_out/s_ops.log 2>&1; rc=$?
echo "=== s_ops rc=$rc $(grep -E 'passed|failed' gpurun_out/s_ops.log | tail -1)"; grep -E "FAILED" gpurun_out/s_ops.log | head
fault gpurun_out/s_ops.log && exit 2; [ $rc -ge 124 ] && exit 1
timeout -k 10 400 env REPLICANN_GEMM_VERBOSE=1 python scripts/decode_bench.py --batches 1,16,64 > gpurun_out/s_decode.log 2>&1; rc=$?
echo "=== decode rc=$rc"; grep '^{' gpurun_out/s_decode.log; grep "gemm tune" gpurun_out/s_decode.log | head -40
[ $rc -ne 0 ] && { tail -5 gpurun_out/s_decode.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_4s -o run -- python3 scripts/decode_bench.py --batches 16 --new 64 > gpurun_out/s_prof.log 2>&1 || { echo "prof failed"; exit 1; }
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_4s/run_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("kernel stats (whole run incl. warm-up generate):", round(tot / 1e6, 2), "ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.3f} ms {int(r["Calls"]):6d} calls  {r["Name"][:110]}')
PY
exit 0
