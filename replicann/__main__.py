"""``python -m replicann train|eval|build [args]`` → :func:`replicann_amd.cli.main`."""
import sys

from replicann_amd.cli import main

sys.exit(main())
