#!/bin/bash
# round 4 (call Z8): K|V cache append fused into the QKV skinny GEMM epilogue: generation GPU tests, decode throughput of
# GPT-2-small at batch 1 / 16 / 64 (eager vs graph-replayed step) and a kernel profile of batch-16 decode.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
fault() { grep -q "illegal memory access\|hipErrorIllegalAddress\|HSA_STATUS_ERROR\|Memory access fault" "$1"; }
PT="python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider"
{ timeout -k 10 300 $PT -x tests/test_ops_gpu.py -k "decode or skinny or linear_kv" && timeout -k 10 300 $PT -x tests/test_generate_gpu.py tests/test_generate.py; } > gpurun_out/z8_gen.log 2>&1; rc=$?
echo "=== z8_gen rc=$rc $(grep -E 'passed|failed' gpurun_out/z8_gen.log | tail -1)"; grep -E "FAILED|Error" gpurun_out/z8_gen.log | head
fault gpurun_out/z8_gen.log && exit 2; [ $rc -ne 0 ] && exit 1
timeout -k 10 400 python scripts/decode_bench.py --batches 1,16,64 > gpurun_out/z8_decode.log 2>&1; rc=$?
echo "=== decode rc=$rc"; grep '^{' gpurun_out/z8_decode.log
[ $rc -ne 0 ] && { tail -5 gpurun_out/z8_decode.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_4z8 -o run -- python3 scripts/decode_bench.py --batches 16 --new 64 > gpurun_out/z8_prof.log 2>&1 || { echo "prof failed"; exit 1; }
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_4z8/run_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("kernel stats (whole run: prefill, eager + graph warm-up and timed generates):", round(tot / 1e6, 2), "ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.3f} ms {int(r["Calls"]):6d} calls  {r["Name"][:110]}')
PY
exit 0
