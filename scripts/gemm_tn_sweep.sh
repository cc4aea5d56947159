# wgrad-layout (tn) vs fwd-layout (nt) main-loop rates at GPT-2-small B=64 wgrad shapes
set -e
for cs in "1 7" "1 4" "8 3" "8 4" "2 4" "6 5" "0 2"; do
  set -- $cs
  python scripts/gemm_one.py 3072 768 65536 tn --cfg $1 --split $2 --iters 10
  python scripts/gemm_one.py 3072 768 65536 nt --cfg $1 --split $2 --iters 10
done
python scripts/gemm_one.py 3072 768 65536 tn --torch --iters 10
python scripts/gemm_one.py 2304 768 65536 tn --iters 10 --split -1
python scripts/gemm_one.py 768 768 65536 tn --iters 10 --split -1
python scripts/gemm_one.py 768 3072 65536 tn --iters 10 --split -1
