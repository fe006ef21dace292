"""UDAF-Hyperopt (reference run_udaf_hyperopt.py)."""

import sys

from .common import run_approach


def main(argv=None):
    return run_approach("udaf", argv, shuffle=False)


if __name__ == "__main__":
    main(sys.argv[1:])
