#!/bin/bash
# round 5 (call U): conv weight-gradient tile variants on the ResNet-18 shapes (scripts/conv_ab.py):
# 2 = 128x192 / 8 waves (default), 4 = 64x192 / 8 waves (new, M = 64 layers), 1 = 64x192 / 4 waves; split target A/B.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_ops_gpu.py -k "conv" > gpurun_out/r5u_tests.log 2>&1; rc=$?
echo "=== tests rc=$rc"; tail -2 gpurun_out/r5u_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for v in 2 4 1; do
  REPLICANN_CONVW=$v timeout -k 10 120 python -u scripts/conv_ab.py > gpurun_out/r5u_v${v}_$r.log 2>&1 || { echo "v$v failed"; tail -3 gpurun_out/r5u_v${v}_$r.log; exit 1; }
  echo "v$v r$r: $(grep conv_wgrad gpurun_out/r5u_v${v}_$r.log | python3 -c 'import sys,json; print(" ".join(str(json.loads(l)["ms"]) for l in sys.stdin))')"
done
REPLICANN_CONVW=4 REPLICANN_CONVW_TARGET=1024 timeout -k 10 120 python -u scripts/conv_ab.py > gpurun_out/r5u_v4t_$r.log 2>&1 || { echo "v4t failed"; exit 1; }
echo "v4 t1024 r$r: $(grep conv_wgrad gpurun_out/r5u_v4t_$r.log | python3 -c 'import sys,json; print(" ".join(str(json.loads(l)["ms"]) for l in sys.stdin))')"
done
