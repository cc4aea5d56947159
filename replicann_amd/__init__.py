"""replicann_amd — MI355X-native (gfx950 / CDNA4) re-design of aaakulchyk/replicann.

Layers:
  nn / arch      reference-compatible attention layers and Transformer blocks
  models         MLP, ResNet-18, GPT-2 small/medium, ViT-B/16
  ops            autograd ops → hand-written HIP kernels (``_C.so``) on GPU, ATen on CPU
  optim          fused flat-buffer AdamW / SGD
  parallel       bucketed RCCL data parallelism
  utils          flat param buffers, synthetic data, checkpoints, metrics
  training       ``train`` / ``evaluate`` entrypoints
"""

from . import arch, models, nn, ops, optim, parallel, utils
from .arch.transformer import TransformerCrossDecoder, TransformerDecoder, TransformerEncoder
from .models import GPT2, MLP, GPT2Config, ResNet18, ViT, ViTConfig
from .nn.attention import (CrossAttentionHead, MultiheadCrossAttention, MultiheadSelfAttention,
                           SelfAttentionHead)
from .training import TrainConfig, Trainer, build_model, evaluate, train

__version__ = "0.1.0"

__all__ = [
    "CrossAttentionHead", "GPT2", "GPT2Config", "MLP", "MultiheadCrossAttention", "MultiheadSelfAttention",
    "ResNet18", "SelfAttentionHead", "TrainConfig", "Trainer", "TransformerCrossDecoder",
    "TransformerDecoder", "TransformerEncoder", "ViT", "ViTConfig", "build_model", "evaluate", "train",
    "arch", "models", "nn", "ops", "optim", "parallel", "utils",
]
