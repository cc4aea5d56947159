"""Rank-0 logging + JSONL metrics and profiling hooks.

``MetricsLogger`` appends one JSON object per logged step (loss, samples/s,
tokens/s, MFU, peak HBM, and the per-phase device milliseconds of that step).
``phase()`` wraps a step phase in a ``torch.profiler.record_function`` range so
``torch.profiler`` / rocprofv3 traces show fwd / bwd / allreduce-wait / optimizer
separately; ``PhaseTimer`` measures the same phases with device events on the
steps that get logged (``allreduce_wait_ms`` = how long the compute stream waited
for the gradient all-reduce after the backward: the exposed communication).
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


class PhaseTimer:
    """Device-event timing of named step phases, only on steps marked active (the event
    records are cheap, the read-back needs one sync, done when the step is logged)."""

    def __init__(self, enabled=True):
        self.enabled = enabled
        self._active = False
        self._paused = 0
        self._ev = []

    @contextlib.contextmanager
    def step(self, active=True):
        self._active = self.enabled and active
        self._ev = []
        try:
            yield
        finally:
            self._active = False

    @contextlib.contextmanager
    def paused(self):  # graph capture / warm-up: no events
        self._paused += 1
        try:
            yield
        finally:
            self._paused -= 1

    @contextlib.contextmanager
    def __call__(self, name):
        if not self._active or self._paused:
            yield
            return
        cuda = torch.cuda.is_available() and torch.cuda.is_initialized()
        if cuda:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            yield
            e.record()
        else:
            s = time.perf_counter()
            yield
            e = time.perf_counter()
        self._ev.append((name, s, e))

    def summary(self):
        """{phase}_ms of the last timed step (summed over micro-batches); {} if none."""
        out = {}
        for name, s, e in self._ev:
            if isinstance(s, float):
                ms = (e - s) * 1e3
            else:
                e.synchronize()
                ms = s.elapsed_time(e)
            out[f"{name}_ms"] = round(out.get(f"{name}_ms", 0.0) + ms, 3)
        self._ev = []
        return out


@contextlib.contextmanager
def phase(name):
    with torch.profiler.record_function(f"replicann::{name}"):
        yield
