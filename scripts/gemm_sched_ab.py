"""A/B of the persistent GEMM's tile schedule on the GPT-2-small step's shapes, in ONE process with
interleaved rounds (guide §5.4 rule 24): static walk vs dynamic queue (and the dynamic queue with a
CU reservation).  Prints one JSON line per (shape, arm): median / min ms and TF/s.

    python scripts/gemm_sched_ab.py [--rounds 5] [--iters 20] [--reserve 0 8 16]
"""

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicann_amd import _ext, ops  # noqa: E402

# (name, M, N, K, layout, act, split)
SHAPES = [
    ("qkv_fwd", 65536, 2304, 768, "nt", 0, 0),
    ("fc_fwd_gelu", 65536, 3072, 768, "nt", 5, 0),
    ("fc2_fwd", 65536, 768, 3072, "nt", 0, 0),
    ("lmhead_fwd", 65536, 50304, 768, "nt", 0, 0),
    ("lmhead_dgrad", 65536, 768, 50304, "nn", 0, 0),
    ("fc_dgrad", 65536, 768, 3072, "nn", 0, 0),
    ("qkv_wgrad_s7", 2304, 768, 65536, "tn", 0, 7),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--reserve", type=int, nargs="*", default=[8])
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    R = _ext.ops()  # loads the native library (fails loudly if missing or stale)
    arms = [("static", 0, 0), ("dynamic", 1, 0)] + [(f"dynamic_r{r}", 1, r) for r in a.reserve]
    for name, M, N, K, lay, act, split in SHAPES:
        if a.only and a.only not in name:
            continue
        ta, tb = lay[0] == "t", lay[1] == "t"
        torch.manual_seed(0)
        A = (torch.rand(*((K, M) if ta else (M, K)), device="cuda") * 2 - 1).bfloat16()
        B = (torch.rand(*((N, K) if tb else (K, N)), device="cuda") * 2 - 1).bfloat16()
        bias = torch.randn(N, device="cuda").bfloat16() if act else None
        pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16) if act else None
        fn = lambda: ops.gemm(A, B, ta=ta, tb=tb, bias=bias, act=act, preact=pre, cfg=9, split_k=split)  # noqa: E731
        times = {arm[0]: [] for arm in arms}
        outs = {}
        for rnd in range(a.rounds):
            for arm, sched, res in arms:
                R.gemm_set_sched(sched)
                R.gemm_set_reserve(res)
                y = fn()
                torch.cuda.synchronize()
                if rnd == 0:
                    outs[arm] = y.clone()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                times[arm].append(e0.elapsed_time(e1) / a.iters)
        R.gemm_set_sched(1)
        R.gemm_set_reserve(0)
        for arm, _, res in arms:
            med = statistics.median(times[arm])
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "layout": lay, "act": act, "split": split,
                              "arm": arm, "ms_median": round(med, 4), "ms_min": round(min(times[arm]), 4),
                              "tflops": round(2 * M * N * K / med / 1e9, 1),
                              "bitwise_equal_static": bool(torch.equal(outs[arm], outs["static"]))}), flush=True)


if __name__ == "__main__":
    main()
