"""Checkpoint save / resume (N26).

* ``model.state_dict()`` is saved unchanged, so R-blocks keep the reference key
  layout (``_attn._heads.{i}._query.weight`` …) and a
  reference-produced state_dict loads with ``strict=True``;
* optimizer state (fp32 master, moments, step), RNG states, step counter and
  a config dict go alongside;
* written by rank 0 only, atomically (tmp file + rename); loading uses
  ``weights_only=True`` and, under DDP, rank 0's parameters are then
  re-broadcast by the DDP wrapper.
"""

from __future__ import annotations

import os

import torch
import torch.distributed as dist


def save_checkpoint(path, model, optimizer=None, step=0, config=None, extra=None):
    if dist.is_initialized() and dist.get_rank() != 0:
        return
    sd = {
        "model": {k: v.detach().cpu() for k, v in model.state_dict().items()},
        "step": int(step),
        "config": dict(config or {}),
        "rng_cpu": torch.get_rng_state(),
    }
    if optimizer is not None:
        sd["optim"] = {k: (v.detach().cpu() if torch.is_tensor(v) else v)
                       for k, v in optimizer.state_dict().items()}
    if extra:
        sd["extra"] = extra
    tmp = f"{path}.tmp"
    torch.save(sd, tmp)
    os.replace(tmp, path)


def load_checkpoint(path, model, optimizer=None, strict=True, map_location="cpu"):
    sd = torch.load(path, map_location=map_location, weights_only=True)
    model.load_state_dict(sd["model"], strict=strict)
    if optimizer is not None and "optim" in sd:
        optimizer.load_state_dict(sd["optim"])
    if "rng_cpu" in sd:
        torch.set_rng_state(sd["rng_cpu"])
    return sd.get("step", 0), sd.get("config", {})
