#!/bin/bash
# round 4 (call Z4, final validation at HEAD (round 4 end: decoding, skinny GEMM, decode attention)): test_ops_gpu.py alone, the rest of the GPU tier, smoke,
# then every BASELINE GPU config's bench (GPT-2-small x2, GPT-2-medium, GPT-2-medium fp8, ViT-B/16,
# ResNet-18).  Any HIP fault ends the call.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
fault() { grep -q "illegal memory access\|hipErrorIllegalAddress\|HSA_STATUS_ERROR\|Memory access fault" "$1"; }
PT="python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PT -x tests/test_ops_gpu.py > gpurun_out/z4_ops.log 2>&1; rc=$?
echo "=== z4_ops rc=$rc $(grep -E 'passed|failed' gpurun_out/z4_ops.log | tail -1)"; grep -E "FAILED" gpurun_out/z4_ops.log | head
fault gpurun_out/z4_ops.log && exit 2; [ $rc -ge 124 ] && exit 1
timeout -k 10 900 $PT tests -m gpu --deselect tests/test_ops_gpu.py > gpurun_out/z4_rest.log 2>&1; rc=$?
echo "=== z4_rest rc=$rc $(grep -E 'passed|failed' gpurun_out/z4_rest.log | tail -1)"; grep -E "FAILED" gpurun_out/z4_rest.log | head
fault gpurun_out/z4_rest.log && exit 2; [ $rc -ge 124 ] && exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/z4_smoke.log 2>&1; echo "=== smoke rc=$? $(grep 'smoke ok' gpurun_out/z4_smoke.log)"
b() {  # b <name> <bench args...>
  local n=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/z4_$n.log 2>&1 || { echo "bench $n failed"; tail -3 gpurun_out/z4_$n.log; exit 1; }
  echo "$n: $(grep '^{' gpurun_out/z4_$n.log | tail -1 | cut -c1-330)"
}
b gpt2s_1 --steps 20 --warmup 5
b gpt2s_2 --steps 20 --warmup 5
b gpt2m --model gpt2-medium --steps 6 --warmup 3
b gpt2m_fp8 --model gpt2-medium-fp8 --steps 6 --warmup 3
b vit --model vit-b16 --steps 8 --warmup 3
b resnet --model resnet18 --steps 20 --warmup 5
b gpt2s_c16k --steps 20 --warmup 5 --ce-chunk 16384
timeout -k 10 400 python scripts/decode_bench.py --batches 1,16,64 > gpurun_out/z4_decode.log 2>&1 || { echo "decode bench failed"; tail -3 gpurun_out/z4_decode.log; exit 1; }
grep '^{' gpurun_out/z4_decode.log | cut -c1-250
exit 0
