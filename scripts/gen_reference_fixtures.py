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
    write_io_floors(tr)


def write_io_floors(tr):
    """The bf16 floors of the stacked encoder → cross-decoder case's OUTPUT and INPUT gradients (the
    reference run in bf16 against itself in fp32), so the GPU test derives those tolerances the way
    it derives the per-parameter ones (1.25 x the reference's own bf16 error) instead of hand-setting
    them.  JSON: plain numbers."""
    import json

    y, gs, gt, _ = _cross(tr, torch.float32)
    y16, gs16, gt16, _ = _cross(tr, torch.bfloat16)
    fl = {refgen.GRAD_CROSS[0]: {"y": _rel(y16, y), "g_src": _rel(gs16, gs), "g_tgt": _rel(gt16, gt)}}
    out = os.path.join(ROOT, "tests", "fixtures", "ref_io_floors.json")
    with open(out, "w") as f:
        json.dump(fl, f, indent=1)
    print(f"wrote {out}: {fl}")


def _rel(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-12))


def _block(tr, cls, H, E, seed, dtype, **kw):
    torch.manual_seed(0)
    m = refgen.zero_dropout(getattr(tr, cls)(H, E, **kw)).train()
    m.load_state_dict(refgen.det_state_dict(m, seed), strict=True)
    m = m.to(dtype)
    if hasattr(m, "_attn_mask"):
        m._attn_mask = m._attn_mask.float()  # the reference accepts only an fp32 mask (quirk Q3)
    return m


def _case(tr, i, dtype):
    name, cls, H, E, T, kw = refgen.GRAD_CASES[i]
    m = _block(tr, cls, H, E, 600 + i, dtype, **kw)
    x = refgen.det_input((2, T, E), 700 + i).to(dtype).requires_grad_()
    y = m(x)
    y.backward(refgen.det_grad(y.shape, 800 + i).to(dtype))
    return y.detach(), x.grad, {n: p.grad for n, p in m.named_parameters()}


def _cross(tr, dtype):
    name, H, E, Ts, Tt = refgen.GRAD_CROSS
    enc = _block(tr, "TransformerEncoder", H, E, 900, dtype)
    dec = _block(tr, "TransformerCrossDecoder", H, E, 901, dtype, context_size=64)
    src = refgen.det_input((2, Ts, E), 902).to(dtype).requires_grad_()
    tgt = refgen.det_input((2, Tt, E), 903).to(dtype).requires_grad_()
    _, k, v = enc(src, return_kv=True)
    y = dec(tgt, k, v)
    y.backward(refgen.det_grad(y.shape, 904).to(dtype))
    grads = {**{"enc." + n: p.grad for n, p in enc.named_parameters()},
             **{"dec." + n: p.grad for n, p in dec.named_parameters()}}
    return y.detach(), src.grad, tgt.grad, grads


def _floor(g32, g16):
    """Per-parameter bf16 floor: the relative L2 error of the REFERENCE's own code run in bf16 (CPU)
    against its fp32 gradients — what "within bf16 tolerance" means for each gradient."""
    return torch.tensor([_rel(g16[n], g32[n]) if g32[n] is not None else 0.0 for n in g32])


def grad_fixtures(tr):
    """Train mode, all dropout at p = 0: outputs, input gradients and EVERY parameter gradient of the
    reference blocks (the native optimizer consumes the parameter gradients, through the fused-QKV
    flat-buffer views), plus each gradient's bf16 floor (the reference itself evaluated in bf16)."""
    fx = {}
    for i, (name, cls, H, E, T, kw) in enumerate(refgen.GRAD_CASES):
        y, gx, g32 = _case(tr, i, torch.float32)
        _, _, g16 = _case(tr, i, torch.bfloat16)
        fx[name] = {"y": y.half(), "gx": gx.half(),
                    "params": {n: (g.half() if g is not None else torch.empty(0)) for n, g in g32.items()},
                    "floor_names": list(g32), "floor": _floor(g32, g16)}
    name = refgen.GRAD_CROSS[0]
    y, gs, gt, g32 = _cross(tr, torch.float32)
    _, _, _, g16 = _cross(tr, torch.bfloat16)
    fx[name] = {"y": y.half(), "g_src": gs.half(), "g_tgt": gt.half(),
                "params": {n: (g.half() if g is not None else torch.empty(0)) for n, g in g32.items()},
                "floor_names": list(g32), "floor": _floor(g32, g16)}
    return fx


if __name__ == "__main__":
    if sys.argv[1:] == ["--io-floors"]:  # only the small JSON (the .pt fixtures stay byte for byte)
        write_io_floors(load_reference())
    else:
        main()
