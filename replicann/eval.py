"""``python -m replicann.eval --model gpt2-small [--checkpoint ckpt.pt]``: evaluation CLI.

Run as a module only; the ``replicann.evaluate(...)`` function is the package attribute."""
from replicann_amd.training import eval_main

if __name__ == "__main__":
    eval_main()
