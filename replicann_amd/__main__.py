"""``python -m replicann_amd train|eval|build [args]`` → :func:`replicann_amd.cli.main`."""
import sys

from .cli import main

sys.exit(main())
