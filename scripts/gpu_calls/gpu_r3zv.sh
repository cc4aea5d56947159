#!/bin/bash
# round 3 (session 2): confirm the non-temporal store threshold 1024 MiB (new default) vs 256 / 4096, three rounds
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "=== $n rc=$rc"; grep -v "amdgpu.ids" gpurun_out/$n.log | grep -o '"ms_per_step": [0-9.]*\|"v2_ms": [0-9.]*' | tail -1; grep -E "passed|failed" gpurun_out/$n.log | tail -1
  return $rc
}
step t_gemm 300 python -u -m pytest tests/test_ops_gpu.py -q -k "gemm or linear" --timeout 120 --timeout-method thread -p no:cacheprovider -x || exit 1
for r in 1 2 3; do
  step g_1024_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
  REPLICANN_GEMM_ST_NT_MB=256 step g_256_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
  REPLICANN_GEMM_ST_NT_MB=8192 step g_8192_$r 300 python bench.py --steps 10 --warmup 3 || exit 1
done
step v_1024 300 python bench.py --model vit-b16 --steps 10 --warmup 3 || exit 1
REPLICANN_GEMM_ST_NT_MB=256 step v_256 300 python bench.py --model vit-b16 --steps 10 --warmup 3 || exit 1
step m_1024 400 python bench.py --model gpt2-medium --steps 5 --warmup 2 || exit 1
REPLICANN_GEMM_ST_NT_MB=256 step m_256 400 python bench.py --model gpt2-medium --steps 5 --warmup 2 || exit 1
