"""CTQ-Hyperopt (reference run_ctq_hyperopt.py)."""

import sys

from .common import run_approach


def main(argv=None):
    return run_approach("ctq", argv, shuffle=False)


if __name__ == "__main__":
    main(sys.argv[1:])
