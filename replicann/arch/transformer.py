"""Alias of :mod:`replicann_amd.arch.transformer` (reference import path)."""
from replicann_amd.arch.transformer import *  # noqa: F401,F403
from replicann_amd.arch.transformer import (_TransformerBlock, _TransformerFFN,  # noqa: F401
                                            TransformerCrossDecoder, TransformerDecoder,
                                            TransformerEncoder)
