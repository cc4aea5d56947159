#!/bin/bash
# round 4 (call J, validation at HEAD): test_ops_gpu.py alone, then the rest of the GPU tier, smoke,
# GPT-2-small bench x2 and a step profile.  Any HIP fault ends the call.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
fault() { grep -q "illegal memory access\|hipErrorIllegalAddress\|HSA_STATUS_ERROR\|Memory access fault" "$1"; }
PT="python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PT -x tests/test_ops_gpu.py > gpurun_out/j_ops.log 2>&1; rc=$?
echo "=== j_ops rc=$rc $(grep -E 'passed|failed' gpurun_out/j_ops.log | tail -1)"; grep -E "FAILED" gpurun_out/j_ops.log | head
fault gpurun_out/j_ops.log && exit 2; [ $rc -ge 124 ] && exit 1
timeout -k 10 900 $PT tests -m gpu --deselect tests/test_ops_gpu.py > gpurun_out/j_rest.log 2>&1; rc=$?
echo "=== j_rest rc=$rc $(grep -E 'passed|failed' gpurun_out/j_rest.log | tail -1)"; grep -E "FAILED" gpurun_out/j_rest.log | head
fault gpurun_out/j_rest.log && exit 2; [ $rc -ge 124 ] && exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/j_smoke.log 2>&1; echo "=== smoke rc=$? $(grep 'smoke ok' gpurun_out/j_smoke.log)"
for r in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/j_bench_$r.log 2>&1 || { echo "bench failed"; exit 1; }
  echo "bench r$r: $(grep '^{' gpurun_out/j_bench_$r.log | tail -1)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_4j -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/j_prof.log 2>&1 || { echo "prof failed"; exit 1; }
python scripts/prof_steps.py gpurun_out/prof_4j/run_kernel_trace.csv --steps 3 > gpurun_out/prof_4j_steps.txt 2>&1
head -24 gpurun_out/prof_4j_steps.txt
exit 0
