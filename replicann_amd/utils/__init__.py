"""Runtime utilities: flat buffers, synthetic data, checkpoints, metrics."""

from .checkpoint import load_checkpoint, save_checkpoint
from .data import SyntheticImages, SyntheticLM, SyntheticMNIST
from .flat import FlatParams
from .metrics import MetricsLogger, phase

__all__ = ["FlatParams", "MetricsLogger", "SyntheticImages", "SyntheticLM", "SyntheticMNIST",
           "load_checkpoint", "phase", "save_checkpoint"]
