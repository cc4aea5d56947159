"""``python -m replicann_amd [train args...]`` → training entrypoint."""
from .training import main

main()
