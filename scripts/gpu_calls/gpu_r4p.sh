#!/bin/bash
# round 4 (call P): LM head + cross-entropy over token chunks (verdict r3 missing item 3):
# GPU numerics test, GPT-2-small step A/B (whole batch vs 16,384- and 8,192-token chunks, with
# peak memory), and a kernel breakdown of the chunked step.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc $(grep -v amdgpu.ids gpurun_out/$n.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"peak_mem_gib": [0-9.]*\|"loss_first_last": [^]]*\|passed\|failed' | tr '\n' ' ')"
  return $rc
}
step p_test 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "chunked or xent or cross_entropy" tests/test_determinism_gpu.py || exit 1
for r in 1 2; do
  step p_whole_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
  step p_c16k_$r 300 python bench.py --steps 10 --warmup 3 --ce-chunk 16384 || exit 1
  step p_c8k_$r 300 python bench.py --steps 10 --warmup 3 --ce-chunk 8192 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_4p -o run -- python3 bench.py --steps 3 --warmup 2 --ce-chunk 16384 > gpurun_out/p_prof.log 2>&1 || { echo "prof failed"; exit 1; }
python scripts/prof_steps.py gpurun_out/prof_4p/run_kernel_trace.csv --steps 3 > gpurun_out/prof_4p_steps.txt 2>&1
head -30 gpurun_out/prof_4p_steps.txt | cut -c1-160
exit 0
