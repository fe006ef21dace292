"""Cerebro-standalone-Hyperopt (reference run_filesystem_cerebro_standalone_hyperopt.py)."""

import sys

from .common import run_approach


def main(argv=None):
    return run_approach("cerebro", argv, shuffle=False)


if __name__ == "__main__":
    main(sys.argv[1:])
