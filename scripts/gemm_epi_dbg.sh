set -e
for d in 0 1 2; do
  for K in 768 3072; do
    REPLICANN_GEMM_DBG=$d python scripts/gemm_one.py 65536 3072 $K nt --cfg 1 --iters 20
  done
done
