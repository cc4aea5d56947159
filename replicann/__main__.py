"""``python -m replicann [train args...]`` → the training entrypoint (replicann_amd.training.main)."""
from replicann_amd.training import main

main()
