"""fp8 backward GEMM A/B on GPT-2-medium shapes (T tokens): the bf16 data / weight gradients the
step runs today vs the fp8 ones (csrc/kernels/fp8.hip rn_gemm_fp8_dgrad / rn_gemm_fp8_wgrad),
plus the one e5m2 quantisation of dY they share.  Interleaved rounds in one process, min per
variant; one JSON line per shape.

    python scripts/fp8_bwd_ab.py [tokens=16384] [rounds=3]
"""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicann_amd import ops  # noqa: E402


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(iters):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / iters


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    torch.manual_seed(0)
    E = 1024
    for name, out_f, in_f in (("qkv", 3 * E, E), ("proj", E, E), ("fc1", 4 * E, E), ("fc2", E, 4 * E)):
        dy = torch.randn(T, out_f, device="cuda", dtype=torch.bfloat16) * 0.01
        x = torch.randn(T, in_f, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(out_f, in_f, device="cuda", dtype=torch.bfloat16) * 0.02
        x8, xs = ops.quantize_fp8(x)
        w8, ws = ops.quantize_fp8(w)
        gs = torch.zeros(4, device="cuda")
        dy8 = torch.ops.replicann.bf8_quantize(dy, gs, False)
        gw = torch.zeros(out_f, in_f, device="cuda", dtype=torch.bfloat16)
        fns = {
            "dgrad_bf16": lambda: ops.gemm(dy, w),
            "dgrad_fp8": lambda: torch.ops.replicann.gemm_fp8_dgrad(dy8, w8, gs, ws, True),
            "wgrad_bf16": lambda: ops.gemm(dy, x, ta=True, split_k=-1, out=gw, accumulate=True),
            "wgrad_fp8": lambda: torch.ops.replicann.gemm_fp8_wgrad(dy8, x8, gs, xs, gw, True, True),
            "quant_dy": lambda: torch.ops.replicann.bf8_quantize(dy, gs, True),
        }
        t = {k: [] for k in fns}
        for _ in range(rounds):
            for k, f in fns.items():
                t[k].append(timeit(f))
        ms = {k: min(v) for k, v in t.items()}
        fl = 2 * T * out_f * in_f
        r = dict(shape=name, T=T, out=out_f, inp=in_f, **{f"{k}_ms": round(v, 4) for k, v in ms.items()},
                 **{f"{k}_tflops": round(fl / ms[k] / 1e9) for k in fns if k != "quant_dy"},
                 bwd_speedup=round((ms["dgrad_bf16"] + ms["wgrad_bf16"])
                                   / (ms["dgrad_fp8"] + ms["wgrad_fp8"] + ms["quant_dy"]), 3))
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
