"""Command-line entrypoints (N21): ``python -m replicann <command> [args]`` (also the
``replicann`` console script installed by pyproject.toml).

    replicann train --model gpt2-small --batch-size 64 --steps 100 [--checkpoint ck.pt]
    replicann eval  --model gpt2-small --checkpoint ck.pt
    replicann generate --model gpt2-small --checkpoint ck.pt --prompt 464,2068 --new 32 --top-k 50
    replicann build            # compile the gfx950 extension in-tree (hipcc --offload-arch=gfx950)
    replicann <train args...>  # no command: train (kept for ``python -m replicann --model ...``)

Sub-commands rather than ``replicann.train`` / ``replicann.eval`` MODULES: a submodule of that
name would replace the ``replicann.train(...)`` function attribute the moment anything imported
it (round-1 API bug), so the package has no such modules.  Launch data-parallel runs under
``python -m torch.distributed.run --nproc-per-node N -m replicann train ...`` (one rank per GPU).
"""

from __future__ import annotations

import sys

COMMANDS = ("train", "eval", "generate", "build")


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    cmd = argv[0] if argv and argv[0] in COMMANDS else "train"
    if argv and argv[0] in COMMANDS:
        argv = argv[1:]
    if cmd == "build":
        from . import _build
        _build.build(verbose=True)
        return 0
    from .training import eval_main, generate_main, main as train_main
    {"eval": eval_main, "generate": generate_main}.get(cmd, train_main)(argv)
    return 0


if __name__ == "__main__":
    sys.exit(main())
