"""Source-compatibility package: ``import replicann`` / ``replicann.nn.attention`` /
``replicann.arch.transformer`` resolve to the MI355X-native implementation in
``replicann_amd`` (same classes, not copies)."""

from replicann_amd import *  # noqa: F401,F403
from replicann_amd import __all__  # noqa: F401
