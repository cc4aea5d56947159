"""Rank-0 logging + JSONL metrics and profiling hooks.

``MetricsLogger`` appends one JSON object per logged step (loss, samples/s,
tokens/s, MFU, peak HBM).  ``phase()`` wraps a step phase in a
``torch.profiler.record_function`` range so ``torch.profiler`` / rocprofv3
traces show fwd / bwd / allreduce-wait / optimizer separately.
"""

from __future__ import annotations

import contextlib
import json
import logging
import time

import torch
import torch.distributed as dist

log = logging.getLogger("replicann")

BF16_PEAK_FLOPS = 2.5e15  # MI355X dense bf16 (MI355X_MICROARCH.md, chip parameters)


def is_rank0():
    return not dist.is_initialized() or dist.get_rank() == 0


class MetricsLogger:
    def __init__(self, path=None):
        self.path = path
        self.t0 = time.time()

    def log(self, **kv):
        if not is_rank0():
            return
        kv.setdefault("wall_s", round(time.time() - self.t0, 3))
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            kv.setdefault("peak_hbm_gb", round(torch.cuda.max_memory_allocated() / 2**30, 2))
        line = json.dumps(kv)
        log.info(line)
        if self.path:
            with open(self.path, "a") as f:
                f.write(line + "\n")


@contextlib.contextmanager
def phase(name):
    with torch.profiler.record_function(f"replicann::{name}"):
        yield
