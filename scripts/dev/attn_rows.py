"""Debug: per-row error of attention outputs / gradients vs fp32 reference (prints rows above tol)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from replicann_amd import ops  # noqa: E402

B, T, H, D = 1, int(sys.argv[1]) if len(sys.argv) > 1 else 128, 1, 64
causal = (sys.argv[2] != "0") if len(sys.argv) > 2 else True
torch.manual_seed(6)
q, k, v = [torch.randn(B, T, H, D, device="cuda").bfloat16() for _ in range(3)]
qg, kg, vg = [t.clone().requires_grad_() for t in (q, k, v)]
o = ops.attention(qg, kg, vg, scale=0.125, causal=causal)
go = torch.randn(B, T, H, D, device="cuda").bfloat16()
o.backward(go)
qf, kf, vf = [t.detach().float().requires_grad_() for t in (q, k, v)]
of = ops.attention_reference(qf, kf, vf, 0.125, causal, None)
of.backward(go.float())
for name, a, b in (("o", o, of), ("dq", qg.grad, qf.grad), ("dk", kg.grad, kf.grad), ("dv", vg.grad, vf.grad)):
    a, b = a.float()[0, :, 0], b.float()[0, :, 0]
    err = (a - b).norm(dim=1) / (b.norm(dim=1) + 1e-3)
    bad = (err > 0.05).nonzero().flatten().tolist()
    print(name, "rel", round(((a - b).norm() / b.norm()).item(), 4), "bad rows", len(bad), bad[:40])
    if bad:
        r = bad[0]
        print("  row", r, "got", a[r, :6].tolist(), "ref", b[r, :6].tolist())
