"""Primitive layers (reference ``src/replicann/nn``)."""

from .attention import (CrossAttentionHead, MultiheadCrossAttention, MultiheadSelfAttention,
                        SelfAttentionHead)

__all__ = ["CrossAttentionHead", "MultiheadCrossAttention", "MultiheadSelfAttention", "SelfAttentionHead"]
