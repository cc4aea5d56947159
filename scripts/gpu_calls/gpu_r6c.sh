#!/bin/bash
# round 6 call C: the 32x32x16 attention kernels (D = 64) — correctness tests, then timings vs the 16x16x32 ones
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "attention" tests/test_determinism_gpu.py tests/test_reference_parity_gpu.py > gpurun_out/r6c_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r6c_tests.log; [ $rc -eq 0 ] || exit 1
O=gpurun_out/r6c_attn.txt; : > $O
for rnd in 1 2; do for a32 in 1 0; do
  REPLICANN_ATTN32=$a32 timeout -k 10 120 python3 scripts/attn_ab.py 64 --rounds 3 2>/dev/null | sed "s/^/a32=$a32 /" >> $O || exit 1
  REPLICANN_ATTN32=$a32 timeout -k 10 120 python3 scripts/attn_ab.py 512 --rounds 3 --T 197 --noncausal 2>/dev/null | sed "s/^/a32=$a32 /" >> $O || exit 1
done; done
cat $O
