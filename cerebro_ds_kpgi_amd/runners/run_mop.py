"""UDAF MOP, lock-step rotation (reference run_mop.py)."""

import sys

from .common import run_approach


def main(argv=None):
    return run_approach("udaf", argv, shuffle=True)


if __name__ == "__main__":
    main(sys.argv[1:])
