"""Device-side dropout seeds (graph-capturable stochastic ops).

Every dropout site (standalone dropout, attention-probability dropout) used to draw its seed on
the host (``torch.randint(...).item()``): a host sync per call, and a seed frozen into a captured
hipGraph — so configs with dropout could not be graph-captured, and the reference blocks always
have head dropout 0.1 in train mode.  Now each call launches ``rng_next`` (one
thread: ``out = splitmix64(state); state += γ``) on the stream and hands ``out`` — a 1-element
int64 device tensor — to the kernel, which reads its seed from there; the backward reuses the
same ``out``.  Replaying a captured step therefore draws fresh masks every step, and eager and
graph runs started from the same state produce identical masks.

The per-device state is seeded from torch's CPU generator (``torch.manual_seed`` governs it) and
travels in checkpoints (``state_dict`` / ``load_state_dict``).
"""

from __future__ import annotations

import torch

from .. import _ext

_STATES: dict[int, torch.Tensor] = {}


def _state(device: torch.device) -> torch.Tensor:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    st = _STATES.get(idx)
    if st is None:
        seed = int(torch.randint(0, 2**62, (1,), dtype=torch.int64).item())
        st = torch.tensor([seed], dtype=torch.int64, device=torch.device("cuda", idx))
        _STATES[idx] = st
    return st


def next_seed(device) -> torch.Tensor:
    """A fresh seed as a 1-element int64 tensor on ``device``, drawn on the device's stream."""
    device = torch.device(device)
    st = _state(device)
    out = torch.empty(1, dtype=torch.int64, device=st.device)
    _ext.ops().rng_next(st, out)
    return out


def state_dict() -> dict:
    return {i: s.detach().cpu().clone() for i, s in _STATES.items()}


def load_state_dict(sd: dict) -> None:
    for i, s in sd.items():
        i = int(i)
        dev = torch.device("cuda", i)
        if i in _STATES:
            _STATES[i].copy_(s.to(dev))
        else:
            _STATES[i] = s.to(dev).clone()


def manual_seed(seed: int) -> None:
    """Reset every device stream to a value derived from ``seed`` (tests)."""
    for i, s in _STATES.items():
        s.fill_(int(seed) * 0x9E3779B1 + i)
