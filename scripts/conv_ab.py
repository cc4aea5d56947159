"""Time the ResNet-18 (batch 256) convolution pieces in one process: implicit-GEMM weight
gradients per layer shape, the stem im2col and the stride-2 col2im gathers.

    REPLICANN_CONVW=<variant> python scripts/conv_ab.py [B]

One JSON line per op (min over rounds)."""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicann_amd import _ext  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / iters)
    return best


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    ops = _ext.ops()
    dev = "cuda"
    v = os.environ.get("REPLICANN_CONVW", "auto")
    # (C, OC, HW_in, K, S, P)
    for C, OC, HW, K, S, P in [(64, 64, 56, 3, 1, 1), (64, 128, 56, 3, 2, 1), (128, 128, 28, 3, 1, 1),
                               (256, 256, 14, 3, 1, 1), (512, 512, 7, 3, 1, 1), (64, 128, 56, 1, 2, 0)]:
        x = torch.randn(B, HW, HW, C, device=dev).bfloat16()
        OH = (HW + 2 * P - K) // S + 1
        dy = torch.randn(B * OH * OH, OC, device=dev).bfloat16()
        ms = timeit(lambda: ops.conv_wgrad_implicit(dy, x, K, K, S, P))
        fl = 2 * OC * K * K * C * B * OH * OH
        print(json.dumps(dict(op="conv_wgrad", variant=v, C=C, OC=OC, HW=HW, K=K, S=S, ms=round(ms, 4),
                              tflops=round(fl / ms / 1e9, 1))), flush=True)
    x = torch.randn(B, 224, 224, 3, device=dev).bfloat16()
    ms = timeit(lambda: ops.im2col(x, 7, 7, 2, 3, 152))
    print(json.dumps(dict(op="im2col_stem", ms=round(ms, 4), gbps=round(B * 112 * 112 * 152 * 2 / ms / 1e6, 1))))
    for C, HW, K, S, P in [(64, 56, 3, 2, 1), (64, 56, 1, 2, 0), (256, 14, 3, 2, 1)]:
        OH = (HW + 2 * P - K) // S + 1
        dcols = torch.randn(B * OH * OH, K * K * C, device=dev).bfloat16()
        ms = timeit(lambda: ops.col2im(dcols, B, HW, HW, C, K, K, S, P, K * K * C))
        print(json.dumps(dict(op="col2im", C=C, HW=HW, K=K, S=S, ms=round(ms, 4),
                              gbps=round((dcols.numel() + B * HW * HW * C) * 2 / ms / 1e6, 1))))


if __name__ == "__main__":
    main()
