"""Time one GEMM shape/config in isolation (for rocprofv3 --pmc runs and A/B tests).

    python scripts/gemm_one.py M N K LAYOUT [--cfg C] [--split S] [--iters N] [--torch]

LAYOUT is two letters (n/t) for op(A), op(B) as in microbench.py (nt = fwd x·Wᵀ,
nn = dgrad dY·W, tn = wgrad dYᵀ·X).  Prints one JSON line.
"""

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicann_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("M", type=int)
    ap.add_argument("N", type=int)
    ap.add_argument("K", type=int)
    ap.add_argument("layout")
    ap.add_argument("--cfg", type=int, default=-1)
    ap.add_argument("--split", type=int, default=0)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--torch", action="store_true", help="time torch.matmul (hipBLASLt) instead")
    ap.add_argument("--act", type=int, default=0,
                    help="epilogue: 0 none, 2 GELU + pre-activation store (fc fwd), 4 GELU backward reading it")
    ap.add_argument("--bias", action="store_true")
    ap.add_argument("--res", action="store_true", help="residual epilogue (full-tile operand read)")
    ap.add_argument("--fp8", default=None, help="e4m3 x e4m3 forward GEMM (layout nt) on kernel 0 / 9 / 11")
    ap.add_argument("--reserve", type=int, default=0, help="CUs the persistent kernel leaves idle (<= 128, multiple of 8)")
    a = ap.parse_args()
    if a.reserve:
        from replicann_amd import _ext
        _ext.ops().gemm_set_reserve(a.reserve)
    ta, tb = a.layout[0] == "t", a.layout[1] == "t"
    torch.manual_seed(0)
    A = torch.randn(*((a.K, a.M) if ta else (a.M, a.K)), device="cuda").bfloat16()
    B = torch.randn(*((a.N, a.K) if tb else (a.K, a.N)), device="cuda").bfloat16()
    if a.fp8 is not None:
        os.environ["REPLICANN_FP8_GEMM"] = a.fp8
        qa, sa = ops.quantize_fp8(A)
        qb, sb = ops.quantize_fp8(B)
        bias = torch.randn(a.N, device="cuda").bfloat16() if a.bias else None
        fn = lambda: torch.ops.replicann.gemm_fp8(qa, qb, sa, sb, bias, None, 0, None)  # noqa: E731
    elif a.torch:
        Am, Bm = (A.t() if ta else A), (B.t() if tb else B)
        fn = lambda: Am @ Bm  # noqa: E731
    else:
        bias = torch.randn(a.N, device="cuda").bfloat16() if a.bias else None
        pre = torch.randn(a.M, a.N, device="cuda").bfloat16() if a.act else None
        res = torch.randn(a.M, a.N, device="cuda").bfloat16() if a.res else None
        fn = lambda: ops.gemm(A, B, ta=ta, tb=tb, cfg=a.cfg, split_k=a.split, bias=bias, act=a.act,  # noqa: E731
                              preact=pre, residual=res)
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    print(json.dumps({"M": a.M, "N": a.N, "K": a.K, "layout": a.layout, "cfg": a.cfg, "split": a.split,
                      "torch": a.torch, "fp8": a.fp8, "act": a.act, "res": a.res,
                      "ms": round(ms, 4),
                      "tflops": round(2 * a.M * a.N * a.K / ms / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
