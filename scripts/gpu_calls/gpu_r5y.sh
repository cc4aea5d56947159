#!/bin/bash
# round 5 (call Y): the halo-tile 3x3 conv (conv3x3.hip) for ResNet's 64-channel layers: tests, then ResNet-18 against
# abso/_C_old.so (the tree before this round's conv / BN changes) and with REPLICANN_CONV3X3=0, alternating; breakdown.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_ops_gpu.py -k "conv or batchnorm or pool" tests/test_resnet_join_gpu.py > gpurun_out/r5y_tests.log 2>&1; rc=$?
echo "=== tests rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/r5y_tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  REPLICANN_SO=abso/_C_old.so timeout -k 10 200 python -u bench.py --model resnet18 --steps 20 --warmup 5 > gpurun_out/r5y_old_$r.log 2>&1 || { echo "old failed"; tail -3 gpurun_out/r5y_old_$r.log; exit 1; }
  REPLICANN_CONV3X3=0 timeout -k 10 200 python -u bench.py --model resnet18 --steps 20 --warmup 5 > gpurun_out/r5y_off_$r.log 2>&1 || { echo "off failed"; tail -3 gpurun_out/r5y_off_$r.log; exit 1; }
  timeout -k 10 200 python -u bench.py --model resnet18 --steps 20 --warmup 5 > gpurun_out/r5y_new_$r.log 2>&1 || { echo "new failed"; tail -3 gpurun_out/r5y_new_$r.log; exit 1; }
  echo "r$r old: $(grep -o '"value": [0-9.]*' gpurun_out/r5y_old_$r.log)  conv3x3 off: $(grep -o '"value": [0-9.]*' gpurun_out/r5y_off_$r.log)  new: $(grep -o '"value": [0-9.]*' gpurun_out/r5y_new_$r.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_5y -o run -- python3 bench.py --model resnet18 --steps 5 --warmup 2 > gpurun_out/r5y_prof.log 2>&1 || { echo "prof failed"; exit 1; }
python scripts/prof_steps.py gpurun_out/prof_5y/run_kernel_trace.csv --steps 5 > gpurun_out/r5y_steps_resnet.txt 2>&1
rm -rf gpurun_out/prof_5y
head -16 gpurun_out/r5y_steps_resnet.txt | cut -c1-150
