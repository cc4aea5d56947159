"""Time the stem im2col (256x224x224x3, 7x7 s2 p3 -> 152-wide cols) on the GPU."""
import os, sys, json
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from replicann_amd import _ext
x = torch.randn(256, 224, 224, 3, device="cuda").bfloat16()
op = _ext.ops().im2col
for _ in range(3):
    op(x, 7, 7, 2, 3, 152)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    op(x, 7, 7, 2, 3, 152)
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 20
gb = 256 * 112 * 112 * 152 * 2 / 1e9
print(json.dumps({"op": "im2col_stem", "ms": round(ms, 4), "write_TBps": round(gb / ms, 2)}))
