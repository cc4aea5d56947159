"""Replicated model families (N17–N20)."""

from .gpt2 import GPT2, GPT2Config
from .mlp import MLP
from .refblock_lm import RefBlockLM, RefBlockLMConfig
from .resnet import ResNet18
from .vit import ViT, ViTConfig

__all__ = ["GPT2", "GPT2Config", "MLP", "RefBlockLM", "RefBlockLMConfig", "ResNet18", "ViT", "ViTConfig"]
