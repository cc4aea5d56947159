"""Communication windows: points in the backward where no persistent GEMM runs.

The persistent 256x256 GEMM (csrc/include/gemm_pk.h) holds every CU with one 512-thread, 128 KiB-LDS,
~250-VGPR workgroup, so a collective whose workgroups sit on some CUs while such a GEMM runs delays
the GEMM's workgroups bound to those CUs for as long as the collective lasts: measured with the comm
proxy, a bucketed all-reduce issued as soon as its gradients exist costs MORE than the same bytes
issued after the backward (profiles/ddp_window_proxy_r3ze.txt).  The attention backward kernels are
ordinary grids of short workgroups that a high-priority collective's workgroups interleave with, so the
data-parallel reducer (``parallel/ddp.py``, ``schedule="window"``) queues ready buckets and issues them
when a window opens: the attention backward calls :func:`open_window` right before its kernels.
"""

from __future__ import annotations

import weakref

_HOOKS: list = []  # weak references to bound methods: a discarded reducer drops out by itself


def register(method):
    _HOOKS.append(weakref.WeakMethod(method))
    return method


def open_window():
    """Called by kernels that leave CUs to a concurrent collective, right before they launch."""
    live = []
    for ref in _HOOKS:
        fn = ref()
        if fn is not None:
            live.append(ref)
            fn()
    _HOOKS[:] = live
