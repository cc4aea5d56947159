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


if __name__ == "__main__":
    main()
