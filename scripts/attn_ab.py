"""A/B the attention kernel variants in ONE process (interleaved rounds, random data):
GPT-2-small shapes (H=12, T=1024, D=64, causal), batch from argv (default 64).

    python scripts/attn_ab.py [B] [--fwd 1,2,3] [--bwd 1,2]

Variants are selected per call through REPLICANN_ATTN_FWD / REPLICANN_ATTN_BWD.  Each
variant's outputs are compared with variant 1's (bitwise-identical math is not required:
max |Δ| is printed).  One JSON line per (pass, variant)."""

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
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("B", type=int, nargs="?", default=64)
    ap.add_argument("--fwd", default="1,2")
    ap.add_argument("--bwd", default="2", help="REPLICANN_ATTN_DQ values (1 or 2 query groups per wave in the dQ kernel)")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--D", type=int, default=64, help="head size (H = 768 // D keeps E = 768)")
    ap.add_argument("--noncausal", action="store_true")
    ap.add_argument("--T", type=int, default=1024, help="sequence length (ViT-B/16: 197, non-causal)")
    a = ap.parse_args()
    B, T, D = a.B, a.T, a.D
    H = 768 // D
    torch.manual_seed(0)
    qkv = torch.randn(B, T, 3, H, D, device="cuda", dtype=torch.bfloat16).requires_grad_()
    go = torch.randn(B, T, H, D, device="cuda", dtype=torch.bfloat16)
    fl_f = 4 * B * H * T * T * D / (1 if a.noncausal else 2)
    fv = [int(x) for x in a.fwd.split(",") if x]
    bv = [int(x) for x in a.bwd.split(",") if x]
    ref_o = ref_g = None
    res = {}
    for rnd in range(a.rounds):
        for v in fv:
            os.environ["REPLICANN_ATTN_FWD"] = str(v)
            f = lambda: ops.attention_packed(qkv, causal=not a.noncausal)
            t = timeit(f)
            o = f().detach()
            if ref_o is None:
                ref_o = o
            err = (o.float() - ref_o.float()).abs().max().item()
            res.setdefault(("fwd", v), []).append((t, err))
        os.environ["REPLICANN_ATTN_FWD"] = "1"
        out = ops.attention_packed(qkv, causal=not a.noncausal)
        for v in bv:
            os.environ["REPLICANN_ATTN_DQ"] = str(v)
            f = lambda: torch.autograd.grad(out, qkv, go, retain_graph=True)[0]
            t = timeit(f)
            gq = f()
            if ref_g is None:
                ref_g = gq
            err = (gq.float() - ref_g.float()).abs().max().item()
            res.setdefault(("bwd", v), []).append((t, err))
    for (ps, v), lst in sorted(res.items()):
        ms = min(x[0] for x in lst)
        fl = fl_f if ps == "fwd" else 2.5 * fl_f
        print(json.dumps(dict(op=f"attn_{ps}", variant=v, B=B, H=H, T=T, D=D, ms=round(ms, 4), tflops=round(fl / ms / 1e9, 1),
                              all_ms=[round(x[0], 4) for x in lst], max_abs_diff_vs_first=max(x[1] for x in lst))),
              flush=True)


if __name__ == "__main__":
    main()
