"""LayerNorm fwd+bwd at the GPT-2-small B=64 shape (M=65536, E=768), pre-LN block form
(residual pass-through + producer-bias reduction).  One JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicann_amd import ops  # noqa: E402
from replicann_amd.utils.flat import FlatParams  # noqa: E402


def main():
    M, E = int(sys.argv[1]) if len(sys.argv) > 1 else 65536, 768
    torch.manual_seed(0)
    mod = torch.nn.Module()
    mod.w = torch.nn.Parameter(torch.ones(E, device="cuda").bfloat16())
    mod.b = torch.nn.Parameter(torch.zeros(E, device="cuda").bfloat16())
    mod.pb = torch.nn.Parameter(torch.zeros(E, device="cuda").bfloat16())
    flat = FlatParams(mod)
    x = torch.randn(M, E, device="cuda").bfloat16().requires_grad_()
    gy, gh = torch.randn(M, E, device="cuda").bfloat16(), torch.randn(M, E, device="cuda").bfloat16()

    fwd_only = os.environ.get("LN_AB_FWD_ONLY") == "1"

    def step():
        if fwd_only:
            with torch.no_grad():
                ops.layer_norm(x, mod.w, mod.b, 1e-5, return_sum=True, producer_bias=mod.pb)
            return
        y, h = ops.layer_norm(x, mod.w, mod.b, 1e-5, return_sum=True, producer_bias=mod.pb)
        torch.autograd.backward([y, h], [gy, gh])

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        step()
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"op": "ln_fwd" if fwd_only else "ln_fwd_bwd", "M": M, "E": E, "waves": os.environ.get("REPLICANN_LN_BWD_WAVES", "default"),
                      "ms": round(e0.elapsed_time(e1) / 20, 4)}), flush=True)


if __name__ == "__main__":
    main()
