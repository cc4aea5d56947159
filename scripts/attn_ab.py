"""Time the production attention kernels (forward, backward) on GPT-2-small shapes (H=12, T=1024,
D=64, causal by default), batch from argv (default 64), random data, several rounds.

    python scripts/attn_ab.py [B] [--rounds 3] [--D 64] [--T 1024] [--noncausal]

Kernel revisions are compared by building each into its own library (REPLICANN_BUILD_OUT) and
running this script once per library (REPLICANN_SO=...): the outputs' checksums are printed so two
revisions can be checked for bitwise equality.  One JSON line per pass (min over rounds)."""

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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--D", type=int, default=64, help="head size (H = 768 // D keeps E = 768)")
    ap.add_argument("--noncausal", action="store_true")
    ap.add_argument("--T", type=int, default=1024, help="sequence length (ViT-B/16: 197, non-causal)")
    ap.add_argument("--bias-grad", action="store_true",
                    help="the packed QKV projection's bias gradient from the backward kernels (producer_bias)")
    a = ap.parse_args()
    B, T, D = a.B, a.T, a.D
    H = 768 // D
    torch.manual_seed(0)
    qkv = torch.randn(B, T, 3, H, D, device="cuda", dtype=torch.bfloat16).requires_grad_()
    go = torch.randn(B, T, H, D, device="cuda", dtype=torch.bfloat16)
    fl_f = 4 * B * H * T * T * D / (1 if a.noncausal else 2)
    pb = None
    if a.bias_grad:  # the bias must live in a flat gradient buffer for the in-kernel partials
        from replicann_amd.utils.flat import FlatParams
        mod = torch.nn.Module()
        mod.pb = torch.nn.Parameter(torch.zeros(3 * H * D, device="cuda").bfloat16())
        flat = FlatParams(mod)
        flat.zero_grad()
        pb = mod.pb
    fwd = lambda: ops.attention_packed(qkv, causal=not a.noncausal, producer_bias=pb)
    out = fwd()
    bwd = lambda: torch.autograd.grad(out, qkv, go, retain_graph=True)[0]
    res = {"fwd": [], "bwd": []}
    for _ in range(a.rounds):
        res["fwd"].append(timeit(fwd))
        res["bwd"].append(timeit(bwd))
    o, g = fwd().detach(), bwd()
    sums = {"fwd": float(o.float().abs().sum()), "bwd": float(g.float().abs().sum())}
    for ps, lst in res.items():
        ms = min(lst)
        fl = fl_f if ps == "fwd" else 2.5 * fl_f
        print(json.dumps(dict(op=f"attn_{ps}", B=B, H=H, T=T, D=D, causal=not a.noncausal, bias_grad=a.bias_grad,
                              ms=round(ms, 4),
                              tflops=round(fl / ms / 1e9, 1), all_ms=[round(x, 4) for x in lst],
                              abs_sum=sums[ps])), flush=True)


if __name__ == "__main__":
    main()
