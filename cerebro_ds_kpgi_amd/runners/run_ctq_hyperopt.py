"""CTQ-Hyperopt (reference run_ctq_hyperopt.py): batched TPE, one greedy
MOP session per batch of ``--concurrency`` configs."""

import sys

from .common import run_approach


def main(argv=None):
    return run_approach("ctq_hyperopt", argv, shuffle=False)


if __name__ == "__main__":
    main(sys.argv[1:])
