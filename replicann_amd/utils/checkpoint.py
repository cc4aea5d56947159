"""Checkpoint save / resume (N26).

* ``model.state_dict()`` is saved unchanged, so R-blocks keep the reference key
  layout (``_attn._heads.{i}._query.weight`` …) and a
  reference-produced state_dict loads with ``strict=True``;
* optimizer state (fp32 master, moments, step), the step counter and a config dict
  go alongside, plus **every rank's** resume state: CPU and device RNG states and the
  data-stream cursor (``extra["ranks"][r]``), gathered to rank 0 — a data-parallel run
  resumed from a checkpoint then takes exactly the steps the uninterrupted run would;
* written by rank 0 only, atomically (tmp file + rename), bracketed by barriers: no
  rank runs ahead of the save, and no rank proceeds (or re-reads the file) before it
  exists; loading uses ``weights_only=True`` and, under DDP, rank 0's parameters are
  then re-broadcast by the DDP wrapper.
"""

from __future__ import annotations

import os

import torch
import torch.distributed as dist


def _dist():
    return dist.is_available() and dist.is_initialized()


def rank_state(data=None):
    """This rank's resume state: RNGs and the data cursor (if the source exposes one)."""
    st = {"rng_cpu": torch.get_rng_state()}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        st["rng_cuda"] = torch.cuda.get_rng_state()
        from ..ops import rng as dev_rng
        st["rng_dropout"] = {str(k): v for k, v in dev_rng.state_dict().items()}  # device dropout streams
    if data is not None and hasattr(data, "state_dict"):
        st["data"] = data.state_dict()
    return st


def save_checkpoint(path, model, optimizer=None, step=0, config=None, extra=None, data=None):
    """Collective under DDP (every rank must call it): gathers the per-rank resume state and
    rank 0 writes.  ``data``: the rank's data source (for its cursor)."""
    mine = rank_state(data)
    if _dist():
        dist.barrier()
        ranks = [None] * dist.get_world_size()
        dist.all_gather_object(ranks, mine)
        is0 = dist.get_rank() == 0
    else:
        ranks, is0 = [mine], True
    if is0:
        sd = {
            "model": {k: v.detach().cpu() for k, v in model.state_dict().items()},
            "step": int(step),
            "config": dict(config or {}),
            "rng_cpu": mine["rng_cpu"],
            "ranks": ranks,
            "world_size": len(ranks),
        }
        if optimizer is not None:
            sd["optim"] = {k: (v.detach().cpu() if torch.is_tensor(v) else v)
                           for k, v in optimizer.state_dict().items()}
        if extra:
            sd["extra"] = extra
        tmp = f"{path}.tmp.{os.getpid()}"
        torch.save(sd, tmp)
        os.replace(tmp, path)
    if _dist():
        dist.barrier()


def load_checkpoint(path, model, optimizer=None, strict=True, map_location="cpu", restore_rng=True,
                    allow_world_change=False):
    """Returns (step, config, this rank's resume state or None).

    The per-rank resume states (RNGs, data cursor) are only meaningful for the world size that
    saved them: resuming with another world size raises, unless ``allow_world_change`` — then
    the model / optimizer state is restored, a warning is issued, and every rank starts fresh
    per-rank streams (returned state None: the caller reseeds them deterministically by rank)."""
    sd = torch.load(path, map_location=map_location, weights_only=True)
    model.load_state_dict(sd["model"], strict=strict)
    if optimizer is not None and "optim" in sd:
        optimizer.load_state_dict(sd["optim"])
    r = dist.get_rank() if _dist() else 0
    world = dist.get_world_size() if _dist() else 1
    ranks = sd.get("ranks") or []
    saved_world = int(sd.get("world_size", len(ranks) or 1))
    if ranks and saved_world != world:
        msg = (f"checkpoint {path} was saved by {saved_world} rank(s) but is resumed by {world}: the per-rank "
               "RNG states and data cursors do not map onto this world size")
        if not allow_world_change:
            raise RuntimeError(msg + " (pass allow_world_change=True to restore only model/optimizer state)")
        import warnings
        warnings.warn(msg + "; restoring model/optimizer state only, per-rank streams start fresh")
        return sd.get("step", 0), sd.get("config", {}), None
    mine = ranks[r] if r < len(ranks) else None
    if mine is not None and sd.get("extra"):
        mine = dict(mine, extra=sd["extra"])
    if restore_rng:
        cpu = mine["rng_cpu"] if mine is not None else sd.get("rng_cpu")
        if cpu is not None:
            torch.set_rng_state(cpu)
        if mine is not None and "rng_cuda" in mine and torch.cuda.is_available():
            torch.cuda.set_rng_state(mine["rng_cuda"])
        if mine is not None and mine.get("rng_dropout") and torch.cuda.is_available():
            from ..ops import rng as dev_rng
            dev_rng.load_state_dict(mine["rng_dropout"])
    return sd.get("step", 0), sd.get("config", {}), mine
