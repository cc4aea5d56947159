"""A/B of GEMM tile configs on the GPT-2 training shapes at a given token count (default
B=64 x T=1024 = 65536 rows), interleaved rounds in one process (MI355X guide §5.4 rule 24),
random bf16 operands.  The vendor library (torch.matmul -> hipBLASLt) is timed as a reference
point only.  One JSON line per shape; writes gpurun_out/gemm_cfg_ab.jsonl.

    python scripts/gemm_cfg_ab.py [--tokens 65536] [--cfgs 9,1,6] [--rounds 3] [--shapes fwd,dgrad,wgrad]
"""

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicann_amd import ops  # noqa: E402


def timeit(fn, iters=10):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=65536)
    ap.add_argument("--cfgs", default="9,1,6")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shapes", default="fwd,dgrad,wgrad")
    ap.add_argument("--E", type=int, default=768)
    ap.add_argument("--V", type=int, default=50304)
    a = ap.parse_args()
    M, E, V = a.tokens, a.E, a.V
    shapes = []
    if "fwd" in a.shapes:
        shapes += [("qkv_fwd", M, 3 * E, E, "nt", 0), ("proj_fwd", M, E, E, "nt", 0),
                   ("fc_fwd_gelu", M, 4 * E, E, "nt", 2), ("fc2_fwd", M, E, 4 * E, "nt", 0),
                   ("lmhead_fwd", M, V, E, "nt", 0)]
    if "dgrad" in a.shapes:
        shapes += [("qkv_dgrad", M, E, 3 * E, "nn", 0), ("proj_dgrad", M, E, E, "nn", 0),
                   ("fc2_dgrad_gelubwd", M, 4 * E, E, "nn", 4), ("fc_dgrad", M, E, 4 * E, "nn", 0),
                   ("lmhead_dgrad", M, E, V, "nn", 0)]
    if "wgrad" in a.shapes:
        shapes += [("qkv_wgrad", 3 * E, E, M, "tn", 0), ("fc_wgrad", 4 * E, E, M, "tn", 0),
                   ("fc2_wgrad", E, 4 * E, M, "tn", 0), ("proj_wgrad", E, E, M, "tn", 0),
                   ("lmhead_wgrad", V, E, M, "tn", 0)]
    cfgs = [int(c) for c in a.cfgs.split(",")]
    os.makedirs("gpurun_out", exist_ok=True)
    out = open("gpurun_out/gemm_cfg_ab.jsonl", "a")
    torch.manual_seed(0)
    for name, m, n, k, lay, act in shapes:
        ta, tb = lay[0] == "t", lay[1] == "t"
        A = torch.randn(*((k, m) if ta else (m, k)), device="cuda").bfloat16()
        B = torch.randn(*((n, k) if tb else (k, n)), device="cuda").bfloat16() * 0.05
        pre = torch.randn(m, n, device="cuda").bfloat16() if act else None
        bias = torch.randn(n, device="cuda").bfloat16() if act == 2 else None
        Am, Bm = (A.t() if ta else A), (B.t() if tb else B)
        ref = (Am.float() @ Bm.float()) if m * n * k < 3e12 else None
        split = -1 if ta else 0
        res = {c: [] for c in cfgs}
        res["lib"] = []
        errs = {}
        for c in cfgs:
            o = ops.gemm(A, B, ta=ta, tb=tb, cfg=c, split_k=split, act=act if act == 2 else 0, bias=bias,
                         preact=pre if act == 2 else None) if act != 4 else torch.ops.replicann.gemm(
                A, B, False, False, None, None, 4, pre, None, False, 0, False, None, c, None)
            if ref is not None and act == 0:
                errs[c] = round(((o.float() - ref).norm() / ref.norm()).item(), 5)
        for _ in range(a.rounds):
            for c in cfgs:
                if act == 4:
                    fn = lambda c=c: torch.ops.replicann.gemm(A, B, False, False, None, None, 4, pre, None, False, 0,  # noqa: E731
                                                              False, None, c, None)
                else:
                    fn = lambda c=c: ops.gemm(A, B, ta=ta, tb=tb, cfg=c, split_k=split, act=act, bias=bias,  # noqa: E731
                                              preact=pre)
                res[c].append(timeit(fn))
            res["lib"].append(timeit(lambda: Am @ Bm))
        fl = 2.0 * m * n * k
        row = {"shape": name, "M": m, "N": n, "K": k, "layout": lay, "act": act,
               "tflops": {str(c): round(fl / min(v) / 1e9, 1) for c, v in res.items()},
               "ms": {str(c): round(min(v), 4) for c, v in res.items()}, "rel_err": errs}
        print(json.dumps(row), flush=True)
        out.write(json.dumps(row) + "\n")


if __name__ == "__main__":
    main()
