"""Architecture blocks (reference ``src/replicann/arch``)."""

from .transformer import TransformerCrossDecoder, TransformerDecoder, TransformerEncoder

__all__ = ["TransformerCrossDecoder", "TransformerDecoder", "TransformerEncoder"]
