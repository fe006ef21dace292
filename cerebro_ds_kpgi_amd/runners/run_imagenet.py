"""MA, model averaging (reference run_imagenet.py)."""

import sys

from .common import run_approach


def main(argv=None):
    return run_approach("ma", argv, shuffle=True)


if __name__ == "__main__":
    main(sys.argv[1:])
