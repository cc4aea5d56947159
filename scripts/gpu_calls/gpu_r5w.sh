#!/bin/bash
# round 5 (call W): ResNet-18 with the 64x192 conv wgrad tile (M = 64) and >= 64-row BN statistics splits, against
# abso/_C_old.so (the tree before both) alternating; conv / BN tests first.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_ops_gpu.py -k "conv or batchnorm or pool" tests/test_resnet_join_gpu.py > gpurun_out/r5w_tests.log 2>&1; rc=$?
echo "=== tests rc=$rc"; tail -2 gpurun_out/r5w_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  REPLICANN_SO=abso/_C_old.so timeout -k 10 200 python -u bench.py --model resnet18 --steps 20 --warmup 5 > gpurun_out/r5w_old_$r.log 2>&1 || { echo "old failed"; tail -3 gpurun_out/r5w_old_$r.log; exit 1; }
  timeout -k 10 200 python -u bench.py --model resnet18 --steps 20 --warmup 5 > gpurun_out/r5w_new_$r.log 2>&1 || { echo "new failed"; tail -3 gpurun_out/r5w_new_$r.log; exit 1; }
  echo "r$r old: $(grep -o '"value": [0-9.]*' gpurun_out/r5w_old_$r.log)  new: $(grep -o '"value": [0-9.]*' gpurun_out/r5w_new_$r.log)"
done
