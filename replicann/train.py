"""``python -m replicann.train --model gpt2-small ...``: the training CLI.

Run as a module only; the ``replicann.train(...)`` function is the package attribute."""
from replicann_amd.training import main

if __name__ == "__main__":
    main()
