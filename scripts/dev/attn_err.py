"""Accuracy of the attention kernels of one library build against fp32 / float64 references, and the
cross-decoder reference-parity errors (tests/test_reference_parity_gpu.py) — to compare two builds
(REPLICANN_SO=...).  One JSON line per case.

    python scripts/dev/attn_err.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from replicann_amd import ops  # noqa: E402


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def attn_case(B, Tq, Tk, H, causal, seed):
    torch.manual_seed(seed)
    q = torch.randn(B, Tq, H, 64, device="cuda").bfloat16()
    k = torch.randn(B, Tk, H, 64, device="cuda").bfloat16()
    v = torch.randn(B, Tk, H, 64, device="cuda").bfloat16()
    go = torch.randn(B, Tq, H, 64, device="cuda").bfloat16()
    qg, kg, vg = [t.clone().requires_grad_() for t in (q, k, v)]
    o = ops.attention(qg, kg, vg, scale=0.125, causal=causal)
    o.backward(go)
    qd, kd, vd = [t.detach().double().requires_grad_() for t in (q, k, v)]
    od = ops.attention_reference(qd, kd, vd, 0.125, causal)
    od.backward(go.double())
    return dict(case=f"attn B{B} Tq{Tq} Tk{Tk} H{H} causal={causal}", o=rel(o, od), dq=rel(qg.grad, qd.grad),
                dk=rel(kg.grad, kd.grad), dv=rel(vg.grad, vd.grad))


def parity_cross():
    import refgen
    import replicann_amd.arch.transformer as T
    fx = torch.load(os.path.join(ROOT, "tests", "fixtures", "ref_gpu_parity.pt"), weights_only=True)
    name, H, E, Ts, Tt = refgen.CROSS
    ref = fx[name]

    def native(cls, seed, **kw):
        torch.manual_seed(0)
        m = getattr(T, cls)(H, E, **kw).eval()
        m.load_state_dict(refgen.det_state_dict(m, seed), strict=True)
        return m.cuda().to(torch.bfloat16)
    enc, dec = native("TransformerEncoder", 500), native("TransformerCrossDecoder", 501, context_size=128)
    src, tgt = refgen.det_input((2, Ts, E), 502), refgen.det_input((2, Tt, E), 503)
    _, k, v = enc(src.cuda().to(torch.bfloat16), return_kv=True)
    ins = [t.detach().cuda().to(torch.bfloat16).requires_grad_() for t in (tgt, k, v)]
    y = dec(*ins)
    y = y[0] if isinstance(y, tuple) else y
    y.backward(refgen.det_grad(y.shape, 504).cuda().to(y.dtype))
    return dict(case="parity cross decoder", y=rel(y, ref["y"]), g_tgt=rel(ins[0].grad, ref["g_tgt"]),
                g_k=rel(ins[1].grad, ref["g_k"]), g_v=rel(ins[2].grad, ref["g_v"]))


if __name__ == "__main__":
    so = os.environ.get("REPLICANN_SO", "tree")
    for args in [(2, 64, 96, 12, False), (2, 64, 64, 12, True), (2, 197, 197, 12, False), (8, 256, 256, 12, False),
                 (2, 100, 260, 12, False), (2, 512, 512, 12, False)]:
        for seed in (1, 2):
            print(json.dumps(dict(so=os.path.basename(so), seed=seed, **attn_case(*args, seed))), flush=True)
    print(json.dumps(dict(so=os.path.basename(so), **parity_cross())), flush=True)
