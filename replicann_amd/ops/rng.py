"""Device-side dropout seeds (graph-capturable stochastic ops).

Every dropout site (standalone dropout, attention-probability dropout) used to draw its seed on
the host (``torch.randint(...).item()``): a host sync per call, and a seed frozen into a captured
hipGraph — so configs with dropout could not be graph-captured, and the reference blocks always
have head dropout 0.1 in train mode.  Now each call launches ``rng_next`` (one
thread: ``out = splitmix64(state); state += γ``) on the stream and hands ``out`` — a 1-element
int64 device tensor — to the kernel, which reads its seed from there; the backward reuses the
same ``out``.  Replaying a captured step therefore draws fresh masks every step, and eager and
graph runs started from the same state produce identical masks.

The per-device state is seeded by ``manual_seed`` (the Trainer passes its run seed and rank), else
from torch's CPU generator, and travels in checkpoints (``state_dict`` / ``load_state_dict``).
"""

from __future__ import annotations

import torch

from .. import _ext

_STATES: dict[int, torch.Tensor] = {}
_BASE: list = [None]  # manual_seed() value: streams created later derive from it too


def _derive(seed: int, idx: int) -> int:
    return (int(seed) * 0x9E3779B1 + idx) & ((1 << 62) - 1)


def _state(device: torch.device) -> torch.Tensor:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    st = _STATES.get(idx)
    if st is None:
        if _BASE[0] is not None:
            seed = _derive(_BASE[0], idx)
        else:
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


def state_tensors(device=None) -> list:
    """The live per-device state tensors (restored in place around graph-capture warm-ups: a
    captured graph holds their addresses); ``device`` creates that device's stream first."""
    if device is not None:
        _state(torch.device(device))
    return list(_STATES.values())


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
    """Reset every device stream (and any created later) to a value derived from ``seed``
    (``Trainer`` calls it with the run's seed, so eager and graph runs draw the same masks)."""
    _BASE[0] = int(seed)
    for i, s in _STATES.items():
        s.fill_(_derive(seed, i))
