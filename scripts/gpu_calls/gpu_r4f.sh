#!/bin/bash
# round 4 (call F): re-run the GPU tests whose tolerances were re-derived and the attention tests, then the staged-epilogue performance pass: M-sweep of the fused-epilogue shapes,
# GPT-2-small step staged vs unstaged, and the step profile at HEAD.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
PT="python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider"
fault() { grep -q "illegal memory access\|hipErrorIllegalAddress\|HSA_STATUS_ERROR\|Memory access fault" "$1"; }
timeout -k 10 300 $PT tests/test_reference_parity_gpu.py tests/test_resnet_join_gpu.py > gpurun_out/t_fixed.log 2>&1; rc=$?
echo "=== t_fixed rc=$rc"; grep -E "passed|failed" gpurun_out/t_fixed.log | tail -1; grep -E "^E   .*Error|FAILED" gpurun_out/t_fixed.log | head
fault gpurun_out/t_fixed.log && exit 2
timeout -k 10 300 $PT tests/test_ops_gpu.py -k "attention" > gpurun_out/t_dkdvp.log 2>&1; rc=$?
echo "=== t_dkdvp rc=$rc"; grep -E "passed|failed" gpurun_out/t_dkdvp.log | tail -1; grep -E "FAILED" gpurun_out/t_dkdvp.log | head
fault gpurun_out/t_dkdvp.log && exit 2
[ $rc -ne 0 ] && exit 1
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc $(grep -v amdgpu.ids gpurun_out/$n.log | grep -o '"value": [0-9.]*, "unit"\|"ms_per_step": [0-9.]*' | tr '\n' ' ')"
  return $rc
}
step msweep 300 python scripts/gemm_msweep.py --m 65536 --staged 0,1 --rounds 3 --shapes proj_fwd,fc2_fwd,fc1_fwd,fc1_dgrad_act6,qkv_fwd || exit 1
grep -v amdgpu.ids gpurun_out/msweep.log | grep '"shape"' | head -40
step msweep_c1 200 python scripts/gemm_msweep.py --m 65536 --cfg 1 --rounds 3 --shapes proj_fwd || exit 1
grep -v amdgpu.ids gpurun_out/msweep_c1.log | grep '"shape"' | head
for r in 1 2; do
  step plain_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
  REPLICANN_GEMM_STAGED=0 step unstaged_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
done
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_4f -o run -- python3 bench.py --steps 3 --warmup 2 || exit 1
python scripts/prof_steps.py gpurun_out/prof_4f/run_kernel_trace.csv --steps 3 > gpurun_out/prof_4f_steps.txt 2>&1
head -30 gpurun_out/prof_4f_steps.txt
exit 0
