# per-tile fixed cost of the GEMM: time vs K at fixed M, N (intercept = prologue + epilogue + launch)
set -e
for K in 384 768 1536 3072 6144; do
  python scripts/gemm_one.py 65536 3072 $K nt --cfg 1 --iters 20
  python scripts/gemm_one.py 65536 3072 $K nt --cfg 2 --iters 20
  python scripts/gemm_one.py 65536 3072 $K nt --torch --iters 20
done
