"""Record the REFERENCE's outputs for the GPU parity tests.

Runs the reference implementation itself — /root/reference/src/replicann, imported read-only —
in fp32 on the CPU with deterministic weights/inputs (tests/refgen.py) and saves its forward
outputs, return_kv tensors and the input gradients of an eval-mode backward to
tests/fixtures/ref_gpu_parity.pt (tensors only, loaded with weights_only=True).  The GPU box has
no /root/reference, so tests/test_reference_parity_gpu.py compares the native bf16 GPU path
against these recorded reference results.

    python scripts/gen_reference_fixtures.py
"""

import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import refgen  # noqa: E402


def load_reference():
    sys.path.insert(0, "/root/reference/src")
    for k in [k for k in sys.modules if k == "replicann" or k.startswith("replicann.")]:
        del sys.modules[k]
    tr = importlib.import_module("replicann.arch.transformer")
    sys.path.remove("/root/reference/src")
    return tr


def fwd_bwd(mod, *inputs, gseed, **kw):
    ins = [t.clone().requires_grad_() for t in inputs]
    out = mod(*ins, **kw)
    y = out[0] if isinstance(out, tuple) else out
    y.backward(refgen.det_grad(y.shape, gseed))
    return y.detach(), [t.grad.detach() for t in ins]


def main():
    tr = load_reference()
    fx = {}
    for i, (name, cls, H, E, T, kw) in enumerate(refgen.CASES):
        torch.manual_seed(0)
        m = getattr(tr, cls)(H, E, **kw).eval()
        m.load_state_dict(refgen.det_state_dict(m, 100 + i), strict=True)
        x = refgen.det_input((2, T, E), 200 + i)
        y, (gx,) = fwd_bwd(m, x, gseed=300 + i)
        fx[name] = {"y": y.half(), "gx": gx.half()}
        if cls == "TransformerEncoder":
            z, k, v = m(x, return_kv=True)
            fx[name].update(kv_z=z.detach().half(), kv_k=k.detach().half(), kv_v=v.detach().half())
    name, H, E, Ts, Tt = refgen.CROSS
    torch.manual_seed(0)
    enc = tr.TransformerEncoder(H, E).eval()
    dec = tr.TransformerCrossDecoder(H, E, context_size=128).eval()
    enc.load_state_dict(refgen.det_state_dict(enc, 500), strict=True)
    dec.load_state_dict(refgen.det_state_dict(dec, 501), strict=True)
    src, tgt = refgen.det_input((2, Ts, E), 502), refgen.det_input((2, Tt, E), 503)
    _, k, v = enc(src, return_kv=True)
    y, (gt, gk, gv) = fwd_bwd(dec, tgt, k.detach(), v.detach(), gseed=504)
    fx[name] = {"y": y.half(), "g_tgt": gt.half(), "g_k": gk.half(), "g_v": gv.half()}
    os.makedirs(os.path.join(ROOT, "tests", "fixtures"), exist_ok=True)
    out = os.path.join(ROOT, "tests", "fixtures", "ref_gpu_parity.pt")
    torch.save(fx, out)
    print(f"wrote {out} ({os.path.getsize(out) / 2**20:.1f} MiB), cases: {sorted(fx)}")
    gx = grad_fixtures(tr)
    out = os.path.join(ROOT, "tests", "fixtures", "ref_gpu_grads.pt")
    torch.save(gx, out)
    print(f"wrote {out} ({os.path.getsize(out) / 2**20:.1f} MiB), cases: {sorted(gx)}")


def param_grads(mod, prefix=""):
    """{state_dict key: .grad} for every parameter (fp16: the fixture travels to the GPU box)."""
    # (a parameter the path does not use — the encoder's _attn._proj under return_kv, quirk Q5 — has
    # no .grad: recorded as an empty tensor, and the native path must not produce one either)
    return {prefix + n: (p.grad.detach().half() if p.grad is not None else torch.empty(0))
            for n, p in mod.named_parameters()}


def grad_fixtures(tr):
    """Train mode, all dropout at p = 0: outputs, input gradients and EVERY parameter gradient of the
    reference blocks (the native optimizer consumes the parameter gradients, through the fused-QKV
    flat-buffer views)."""
    fx = {}
    for i, (name, cls, H, E, T, kw) in enumerate(refgen.GRAD_CASES):
        torch.manual_seed(0)
        m = refgen.zero_dropout(getattr(tr, cls)(H, E, **kw)).train()
        m.load_state_dict(refgen.det_state_dict(m, 600 + i), strict=True)
        x = refgen.det_input((2, T, E), 700 + i)
        y, (g,) = fwd_bwd(m, x, gseed=800 + i)
        fx[name] = {"y": y.half(), "gx": g.half(), "params": param_grads(m)}
    name, H, E, Ts, Tt = refgen.GRAD_CROSS
    torch.manual_seed(0)
    enc = refgen.zero_dropout(tr.TransformerEncoder(H, E)).train()
    dec = refgen.zero_dropout(tr.TransformerCrossDecoder(H, E, context_size=64)).train()
    enc.load_state_dict(refgen.det_state_dict(enc, 900), strict=True)
    dec.load_state_dict(refgen.det_state_dict(dec, 901), strict=True)
    src = refgen.det_input((2, Ts, E), 902).requires_grad_()
    tgt = refgen.det_input((2, Tt, E), 903).requires_grad_()
    _, k, v = enc(src, return_kv=True)
    y = dec(tgt, k, v)
    y.backward(refgen.det_grad(y.shape, 904))
    fx[name] = {"y": y.detach().half(), "g_src": src.grad.half(), "g_tgt": tgt.grad.half(),
                "params": {**param_grads(enc, "enc."), **param_grads(dec, "dec.")}}
    return fx


if __name__ == "__main__":
    main()
