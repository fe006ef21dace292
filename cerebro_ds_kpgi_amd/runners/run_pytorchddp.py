"""PyTorch-DDP baseline (reference run_pytorchddp.py)."""

import sys

from .common import run_approach


def main(argv=None):
    return run_approach("ddp", argv, shuffle=True)


if __name__ == "__main__":
    main(sys.argv[1:])
