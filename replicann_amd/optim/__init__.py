"""Fused flat-buffer optimizers (N12/N13)."""

from .fused import FusedAdamW, FusedSGD, cosine_lr

__all__ = ["FusedAdamW", "FusedSGD", "cosine_lr"]
