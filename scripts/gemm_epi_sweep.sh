set -e
for cfg in 1 6 8 0; do
  python scripts/gemm_one.py 65536 3072 768 nt --cfg $cfg --iters 20
  python scripts/gemm_one.py 65536 3072 768 nt --cfg $cfg --iters 20 --act 2 --bias
  python scripts/gemm_one.py 65536 3072 768 nn --cfg $cfg --iters 20
  python scripts/gemm_one.py 65536 3072 768 nn --cfg $cfg --iters 20 --act 4
done
python scripts/gemm_one.py 65536 3072 768 nt --torch --iters 20
python scripts/gemm_one.py 65536 3072 768 nn --torch --iters 20
