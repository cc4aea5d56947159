#!/bin/bash
# round 3: fused-dQ backward non-causal (no spills) vs two-kernel; BN relu-mask ResNet check
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python scripts/attn_ab.py 64 --fwd 3 --bwd 2,3 --rounds 3 --noncausal > gpurun_out/attn_ab_nc.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/attn_ab_nc.jsonl
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_determinism_gpu.py tests/test_convergence_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "batchnorm or bn or resnet or conv" > gpurun_out/bn_test.log 2>&1
rc=$?; tail -3 gpurun_out/bn_test.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --model resnet18 --steps 20 --warmup 3 > gpurun_out/rn18_mask.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/rn18_mask.log | tail -1 | cut -c1-200; exit $rc
