"""Cerebro standalone over file partitions (reference run_filesystem_cerebro_standalone.py)."""

import sys

from .common import run_approach


def main(argv=None):
    return run_approach("cerebro", argv, shuffle=False)


if __name__ == "__main__":
    main(sys.argv[1:])
