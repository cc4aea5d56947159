#!/bin/bash
# round 3: DDP step beside the comm proxy — static / overlap-only queue, fp32 / bf16 reduction;
# own GEMM vs torch.matmul on the verdict's four headline shapes
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | tail -2 | cut -c1-250
  return $rc
}
step ddp_test 300 python -u -m pytest tests/test_comm_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
for s in "65536 2304 768 nt" "65536 768 3072 nt" "65536 50304 768 nt" "65536 768 50304 nn"; do
  n=$(echo $s | tr ' ' '_')
  step own_$n 120 python scripts/gemm_one.py $s || exit 1
  step lib_$n 120 python scripts/gemm_one.py $s --torch || exit 1
done
step plain 300 python bench.py --steps 10 --warmup 3 || exit 1
step px_static 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy || exit 1
REPLICANN_GEMM_SCHED=overlap step px_overlap 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy || exit 1
step px_static_bf16 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy --reduce-dtype bf16 || exit 1
REPLICANN_GEMM_SCHED=overlap step px_overlap_bf16 300 python bench.py --steps 10 --warmup 3 --ddp on --comm proxy --reduce-dtype bf16 || exit 1
step prof_px_static 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_px_static -o run -- python3 bench.py --steps 3 --warmup 2 --ddp on --comm proxy
