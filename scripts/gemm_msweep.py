"""Time the persistent GEMM over a sweep of M at fixed N, K (per-launch fixed cost vs per-tile
cost: fit t = a + b·tiles_per_CU).  One JSON line per (shape, M).

    python scripts/gemm_msweep.py [--iters 30]
"""

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicann_amd import _ext, ops  # noqa: E402

SHAPES = [  # (name, N, K, layout, act, residual)
    ("proj_fwd", 768, 768, "nt", 0, True),
    ("qkv_fwd", 2304, 768, "nt", 0, False),
    ("fc2_fwd", 768, 3072, "nt", 0, True),
    ("proj_dgrad", 768, 768, "nn", 0, False),
    ("fc1_fwd", 3072, 768, "nt", 5, False),
    ("fc1_dgrad_act6", 3072, 768, "nn", 6, False),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--shapes", default=None, help="comma-separated subset of the shape names")
    ap.add_argument("--m", default="16384,32768,65536,131072,262144")
    ap.add_argument("--cfg", type=int, default=9, help="tile config (9 = persistent; -1 = autotuned pick)")
    ap.add_argument("--rounds", type=int, default=1)
    a = ap.parse_args()
    _ext.ops()  # load the library: torch.ops.replicann.* below are used before any op call
    torch.manual_seed(0)
    for name, N, K, lay, act, res in SHAPES:
        if a.shapes and name not in a.shapes.split(","):
            continue
        for M in map(int, a.m.split(",")):
            ta, tb = lay[0] == "t", lay[1] == "t"
            A = torch.randn(*((K, M) if ta else (M, K)), device="cuda").bfloat16()
            B = torch.randn(*((N, K) if tb else (K, N)), device="cuda").bfloat16()
            R = torch.randn(M, N, device="cuda").bfloat16() if res else None
            pre = (torch.rand(M, N, device="cuda").bfloat16() if act in (3, 4, 6)  # read by the epilogue
                   else torch.empty(M, N, device="cuda", dtype=torch.bfloat16) if act else None)
            fn = lambda: ops.gemm(A, B, ta=ta, tb=tb, residual=R, act=act, preact=pre, cfg=a.cfg)  # noqa: E731
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(a.iters):
                    fn()
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for rnd in range(a.rounds):
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / a.iters
                tiles = -(-M // 256) * -(-N // 256)
                print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "cfg": a.cfg,
                                  "tiles_per_cu": round(tiles / 256, 2), "us": round(ms * 1e3, 2),
                                  "tflops": round(2 * M * N * K / ms / 1e9, 1)}), flush=True)
            del A, B, R, pre, g


if __name__ == "__main__":
    main()
