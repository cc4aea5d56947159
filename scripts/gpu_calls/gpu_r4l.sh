#!/bin/bash
# round 4 (call L): ResNet-18 b256 bench + step profile after the shortcut-gradient join (no ATen add
# expected in the step), the ResNet convergence tests, and the GPT-2-medium fp8 (forward GEMMs only,
# the default fp8 config) 50-step trajectory against bf16.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
fault() { grep -q "illegal memory access\|hipErrorIllegalAddress\|HSA_STATUS_ERROR\|Memory access fault" "$1"; }
PT="python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $PT tests/test_ops_gpu.py tests/test_determinism_gpu.py -k "attention or attn or determin" > gpurun_out/l_attn.log 2>&1; rc=$?
echo "=== l_attn rc=$rc $(grep -E 'passed|failed' gpurun_out/l_attn.log | tail -1)"; grep -E "FAILED" gpurun_out/l_attn.log | head
fault gpurun_out/l_attn.log && exit 2
timeout -k 10 300 $PT tests/test_convergence_gpu.py tests/test_resnet_join_gpu.py -k "resnet or join or block" > gpurun_out/l_tests.log 2>&1; rc=$?
echo "=== l_tests rc=$rc $(grep -E 'passed|failed' gpurun_out/l_tests.log | tail -1)"; grep -E "FAILED" gpurun_out/l_tests.log | head
fault gpurun_out/l_tests.log && exit 2
for r in 1 2; do
  timeout -k 10 300 python bench.py --model resnet18 --steps 20 --warmup 5 > gpurun_out/l_resnet_$r.log 2>&1 || { echo "resnet bench failed"; exit 1; }
  echo "resnet r$r: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/l_resnet_$r.log | tr '\n' ' ')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_4l_resnet -o run -- python3 bench.py --model resnet18 --steps 5 --warmup 3 > gpurun_out/l_prof.log 2>&1 || { echo "prof failed"; exit 1; }
python scripts/prof_steps.py gpurun_out/prof_4l_resnet/run_kernel_trace.csv --steps 5 --marker sgd_k > gpurun_out/prof_4l_resnet_steps.txt 2>&1
head -30 gpurun_out/prof_4l_resnet_steps.txt
timeout -k 10 600 python scripts/fp8_trajectory.py 50 16 1e-4 > gpurun_out/l_traj_m8fwd.log 2>&1; echo "=== traj fp8 fwd rc=$? $(grep summary gpurun_out/l_traj_m8fwd.log)"
exit 0
