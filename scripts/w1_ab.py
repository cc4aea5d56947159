"""A/B of the one-wave-per-SIMD persistent GEMM (cfg 11, csrc/include/gemm_w1.h) against the 8-wave
persistent kernel (cfg 9) and, for fp8, the one-tile-per-block kernel, on the GPT-2 forward shapes
(M = 64 × 1024 tokens), bias epilogue, random operands.  Interleaved rounds in one process (guide
§5.4 rule 24); one JSON line per (shape, kernel) with the best and median round.

    python scripts/w1_ab.py [--rounds 5] [--iters 20] [--only bf16|fp8]
"""

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicann_amd import _ext, ops  # noqa: E402

# (name, N, K, B layout): "nt" = x·Wᵀ (W [N, K]), "nn" = the data gradient dY·W (W [K, N])
BF16 = [("s_qkv", 2304, 768, "nt"), ("s_proj", 768, 768, "nt"), ("s_fc1_plain", 3072, 768, "nt"),
        ("s_fc2", 768, 3072, "nt"), ("m_qkv", 3072, 1024, "nt"), ("m_fc2", 1024, 4096, "nt"),
        ("s_dgrad_qkv", 768, 2304, "nn"), ("s_dgrad_fc1", 768, 3072, "nn"), ("s_dgrad_fc2", 3072, 768, "nn"),
        ("s_dgrad_proj", 768, 768, "nn"), ("s_proj_res", 768, 768, "res"), ("s_fc2_res", 768, 3072, "res"),
        ("m_proj_res", 1024, 1024, "res"), ("m_fc2_res", 1024, 4096, "res")]
FP8 = [("m_qkv", 3072, 1024, False), ("m_proj", 1024, 1024, False), ("m_fc1_plain", 4096, 1024, False),
       ("m_fc2", 1024, 4096, False), ("m_proj_res", 1024, 1024, True), ("m_fc2_res", 1024, 4096, True)]


def graph_time(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()

    def run():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters

    return run


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--m", type=int, default=65536)
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    _ext.ops()
    torch.manual_seed(0)
    M = a.m
    if a.only in (None, "bf16"):
        for name, N, K, lay in BF16:
            x = torch.randn(M, K, device="cuda").bfloat16()
            nt = lay != "nn"
            w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16() if nt else (torch.randn(K, N, device="cuda") * 0.05).bfloat16()
            bias = (torch.randn(N, device="cuda") * 0.1).bfloat16() if nt else None
            res = torch.randn(M, N, device="cuda").bfloat16() if lay == "res" else None
            runs = {cfg: graph_time(lambda cfg=cfg: ops.gemm(x, w, tb=nt, bias=bias, residual=res, cfg=cfg), a.iters)
                    for cfg in (9, 11)}
            t = {cfg: [] for cfg in runs}
            for _ in range(a.rounds):
                for cfg, r in runs.items():
                    t[cfg].append(r())
            fl = 2.0 * M * N * K
            for cfg, v in t.items():
                print(json.dumps({"dtype": "bf16", "shape": name, "layout": lay, "M": M, "N": N, "K": K, "cfg": cfg,
                                  "ms_min": round(min(v), 4), "ms_med": round(statistics.median(v), 4),
                                  "tflops": round(fl / min(v) / 1e9, 1)}), flush=True)
            del runs
    if a.only in (None, "fp8"):
        for name, N, K, with_res in FP8:
            x = torch.randn(M, K, device="cuda").bfloat16()
            w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
            bias = (torch.randn(N, device="cuda") * 0.1).bfloat16()
            qa, sa = ops.quantize_fp8(x)
            qb, sb = ops.quantize_fp8(w)
            res = torch.randn(M, N, device="cuda").bfloat16() if with_res else None
            runs = {}
            for kern in ("0", "9", "11"):
                os.environ["REPLICANN_FP8_GEMM"] = kern
                runs[kern] = graph_time(lambda: torch.ops.replicann.gemm_fp8(qa, qb, sa, sb, bias, res, 0, None), a.iters)
            t = {k: [] for k in runs}
            for _ in range(a.rounds):
                for k, r in runs.items():
                    t[k].append(r())
            fl = 2.0 * M * N * K
            for k, v in t.items():
                print(json.dumps({"dtype": "fp8", "shape": name, "M": M, "N": N, "K": K, "kernel": k,
                                  "ms_min": round(min(v), 4), "ms_med": round(statistics.median(v), 4),
                                  "tflops": round(fl / min(v) / 1e9, 1)}), flush=True)
            del runs
    os.environ.pop("REPLICANN_FP8_GEMM", None)


if __name__ == "__main__":
    main()
