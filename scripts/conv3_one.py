"""Run the ResNet-18 layer-1 convolution (B=256, 56x56x64 -> 64, 3x3 s1 p1) forward (+statistics) and data gradient
a few times on whichever path the library takes (conv3x3.hip halo kernel, or the implicit GEMM with
REPLICANN_CONV3X3=0): a small driver for rocprofv3 --pmc passes.

    python scripts/conv3_one.py [iters]
"""

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicann_amd import _ext  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    o = _ext.ops()
    x = torch.randn(256, 56, 56, 64, device="cuda").bfloat16()
    w = (torch.randn(64, 3, 3, 64, device="cuda") * 0.05).bfloat16()
    dy = torch.randn(256, 56, 56, 64, device="cuda").bfloat16()
    for _ in range(iters):
        o.conv_fwd_implicit_stats(x, w, None, 1, 1)
        o.conv_dgrad_implicit(dy, w, 56, 56, 1)
    torch.cuda.synchronize()
    print("ok", iters)


if __name__ == "__main__":
    main()
