"""Hyperopt task parallel (reference run_hyperopt.py)."""

import sys

from .common import run_approach


def main(argv=None):
    return run_approach("task", argv, shuffle=True)


if __name__ == "__main__":
    main(sys.argv[1:])
