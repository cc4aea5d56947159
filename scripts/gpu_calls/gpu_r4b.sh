#!/bin/bash
# round 4 (call B1, performance): staged vs unstaged GEMM epilogue — sweep, GPT-2-small step A/B,
# PMC — fp8 backward GEMMs (tests, A/B, GPT-2-medium step) and the step profile at HEAD
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | grep -o '"ms_per_step": [0-9.]*' | tail -1
  return $rc
}
step msweep 300 python scripts/gemm_msweep.py --m 65536 --staged 0,1 --rounds 3 --shapes proj_fwd,fc2_fwd,fc1_dgrad_act6,qkv_fwd || exit 1
for r in 1 2; do
  step plain_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
  REPLICANN_GEMM_STAGED=0 step unstaged_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
done
for r in 1 2; do
  REPLICANN_FP8_WGRAD=0 step m8_bf16w_$r 300 python bench.py --model gpt2-medium-fp8 --steps 6 --warmup 3 || exit 1
  REPLICANN_FP8_WGRAD=1 step m8_fp8w_$r 300 python bench.py --model gpt2-medium-fp8 --steps 6 --warmup 3 || exit 1
done
step fp8_bwd_tests 300 python -u -m pytest tests/test_fp8_wgrad_gpu.py -x -v --timeout 120 --timeout-method thread || exit 1
step fp8_bwd_ab 300 python scripts/fp8_bwd_ab.py 16384 3 || exit 1
for r in 1 2; do
  REPLICANN_FP8_WGRAD=1 REPLICANN_FP8_DGRAD=1 step m8_fp8wd_$r 300 python bench.py --model gpt2-medium-fp8 --steps 6 --warmup 3 || exit 1
done
step pmc_staged 600 bash scripts/pmc_staged.sh || exit 1
python scripts/pmc_summary.py gpurun_out/pmc_stg/*_counter_collection.csv --match gemm_pk > gpurun_out/pmc_staged_summary.txt 2>&1
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_4b -o run -- python3 bench.py --steps 3 --warmup 2 || exit 1
python scripts/prof_steps.py gpurun_out/prof_4b/run_kernel_trace.csv --steps 3 > gpurun_out/prof_4b_steps.txt 2>&1
exit 0
