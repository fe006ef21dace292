"""CTQ, greedy work-conserving MOP (reference ctq.py)."""

import sys

from .common import run_approach


def main(argv=None):
    return run_approach("ctq", argv, shuffle=True)


if __name__ == "__main__":
    main(sys.argv[1:])
