"""fp8 forward GEMM A/B on the GPT-2-medium b64 shapes (M = 65536 tokens): the persistent
256x256 fp8 kernel (gemm_pk<..., FP8>, REPLICANN_FP8_GEMM=9, default) vs the one-tile-per-block
256x192 fp8 kernel (=0) vs the autotuned bf16 GEMM, plus the one-pass activation quantisation.
Interleaved in one process; prints one JSON line per shape."""

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
    torch.manual_seed(0)
    M = 64 * 1024
    for name, n, k, act in (("qkv", 3072, 1024, 0), ("proj", 1024, 1024, 0), ("fc1_gelu", 4096, 1024, 5),
                            ("fc2", 1024, 4096, 0)):
        a = torch.randn(M, k, device="cuda", dtype=torch.bfloat16)
        b = torch.randn(n, k, device="cuda", dtype=torch.bfloat16) * 0.05
        bias = torch.randn(n, device="cuda", dtype=torch.bfloat16) * 0.1
        qa, sa = ops.quantize_fp8(a)
        qb, sb = ops.quantize_fp8(b)
        pre = torch.empty(M, n, device="cuda", dtype=torch.bfloat16) if act == 5 else None
        st = sa.clone()
        f8 = lambda: torch.ops.replicann.gemm_fp8(qa, qb, sa, sb, bias, None, act, pre)
        b16 = lambda: ops.gemm(a, b, tb=True, bias=bias, act=act, preact=pre)
        qd = lambda: torch.ops.replicann.fp8_quantize_delayed(a, st)
        fl = 2 * M * n * k
        t = {"fp8_pk": [], "fp8_tile": [], "bf16": [], "quant": []}
        for _ in range(3):
            os.environ["REPLICANN_FP8_GEMM"] = "9"
            t["fp8_pk"].append(timeit(f8))
            os.environ["REPLICANN_FP8_GEMM"] = "0"
            t["fp8_tile"].append(timeit(f8))
            t["bf16"].append(timeit(b16))
            t["quant"].append(timeit(qd))
        os.environ["REPLICANN_FP8_GEMM"] = "9"
        ms = {kk: min(v) for kk, v in t.items()}
        o9 = f8().float()
        os.environ["REPLICANN_FP8_GEMM"] = "0"
        o0 = f8().float()
        os.environ["REPLICANN_FP8_GEMM"] = "9"
        r = dict(shape=name, M=M, N=n, K=k, act=act, **{f"{kk}_ms": round(v, 4) for kk, v in ms.items()},
                 **{f"{kk}_tflops": round(fl / ms[kk] / 1e9) for kk in ("fp8_pk", "fp8_tile", "bf16")},
                 pk_vs_tile_rel=((o9 - o0).norm() / o0.norm()).item())
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
