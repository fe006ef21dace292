"""DA-DDP baseline (reference run_pytorchddp_da.py)."""

import sys

from .common import run_approach


def main(argv=None):
    return run_approach("ddp", argv, shuffle=True)


if __name__ == "__main__":
    main(sys.argv[1:])
