#!/bin/bash
# round 4 (call Z9): closing check of the final tree — every GPU test, smoke, GPT-2-small bench, decode bench.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
fault() { grep -q "illegal memory access\|hipErrorIllegalAddress\|HSA_STATUS_ERROR\|Memory access fault" "$1"; }
PT="python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $PT tests -m gpu > gpurun_out/z9_gpu.log 2>&1; rc=$?
echo "=== z9_gpu rc=$rc $(grep -E 'passed|failed' gpurun_out/z9_gpu.log | tail -1)"; grep -E "FAILED" gpurun_out/z9_gpu.log | head
fault gpurun_out/z9_gpu.log && exit 2; [ $rc -ge 124 ] && exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/z9_smoke.log 2>&1; echo "=== smoke rc=$? $(grep 'smoke ok' gpurun_out/z9_smoke.log)"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/z9_gpt2s.log 2>&1 || { echo "bench failed"; tail -3 gpurun_out/z9_gpt2s.log; exit 1; }
echo "gpt2s: $(grep '^{' gpurun_out/z9_gpt2s.log | cut -c1-330)"
timeout -k 10 400 python scripts/decode_bench.py --batches 1,16,64 > gpurun_out/z9_decode.log 2>&1 || { echo "decode bench failed"; tail -3 gpurun_out/z9_decode.log; exit 1; }
grep '^{' gpurun_out/z9_decode.log | cut -c1-250
exit 0
