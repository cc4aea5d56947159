"""Alias of :mod:`replicann_amd.nn.attention` (reference import path)."""
from replicann_amd.nn.attention import *  # noqa: F401,F403
from replicann_amd.nn.attention import (_AttentionHead, _MultiheadAttention, CrossAttentionHead,  # noqa: F401
                                        MultiheadCrossAttention, MultiheadSelfAttention,
                                        SelfAttentionHead)
