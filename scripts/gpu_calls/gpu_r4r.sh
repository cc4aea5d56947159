#!/bin/bash
# round 4 (call R): GPT-2 KV-cache decoding — GPU tests (cached steps vs the full forward, head sizes
# 64 / 32), decode throughput of GPT-2-small at batch 1 / 16 / 64, and a kernel profile of batch-16 decode.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
PT="python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $PT tests/test_generate_gpu.py tests/test_generate.py > gpurun_out/r_test.log 2>&1; rc=$?
echo "=== r_test rc=$rc $(grep -E 'passed|failed' gpurun_out/r_test.log | tail -1)"; grep FAILED gpurun_out/r_test.log | head
[ $rc -ne 0 ] && exit 1
timeout -k 10 400 python scripts/decode_bench.py --batches 1,16,64 > gpurun_out/r_decode.log 2>&1; rc=$?
echo "=== decode rc=$rc"; grep '^{' gpurun_out/r_decode.log
[ $rc -ne 0 ] && { tail -5 gpurun_out/r_decode.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_4r -o run -- python3 scripts/decode_bench.py --batches 16 --new 64 > gpurun_out/r_prof.log 2>&1 || { echo "prof failed"; exit 1; }
python - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/prof_4r/run_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("kernel stats (whole run incl. warm-up generate):", round(tot / 1e6, 2), "ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.3f} ms {int(r["Calls"]):6d} calls  {r["Name"][:110]}')
PY
exit 0
