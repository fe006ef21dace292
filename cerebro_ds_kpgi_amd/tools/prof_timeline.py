"""One training step's kernel timeline from a rocprofv3 SQLite output.

    python -m cerebro_ds_kpgi_amd.tools.prof_timeline gpurun_out/prof_c1 [--step -2] > t.md

Picks the dispatches between two consecutive fused-Adam kernels (one per
step; ``--step -2`` = the last complete step) and prints, in start order:
kernel (short name), grid / workgroup size, duration, and the idle gap to
the previous dispatch's end on any stream.  The footer splits the step wall
time into kernel-busy time and gaps, and lists the top kernels by time.
What a step of a latency-bound config spends between kernels (launch
floor, dependency waits) versus inside them is the question this answers.
"""

import argparse
import re
import sqlite3

from .prof_summary import find_db


def _short(name):
    n = re.sub(r"\(.*$", "", name)
    n = re.sub(r"^void ", "", n)
    return n[:70]


def _cols(con):
    cur = con.execute("select * from kernels limit 1")
    return [d[0] for d in cur.description]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--step", type=int, default=-2,
                    help="which Adam-delimited step (python index over complete steps)")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    con = sqlite3.connect(find_db(a.path))
    cols = _cols(con)
    want = ["name", "start", "end"]
    extra = [c for c in cols if re.search(r"grid_size|workgroup_size|^grid|^workgroup", c, re.I)]
    rows = list(con.execute("select {} from kernels order by start".format(
        ", ".join(want + extra))))
    ends = [i for i, r in enumerate(rows) if "adam_kernel" in r[0]]
    if len(ends) < 2:
        raise SystemExit("need at least two Adam dispatches, found {}".format(len(ends)))
    bounds = list(zip(ends[:-1], ends[1:]))
    i0, i1 = bounds[a.step]
    step = rows[i0 + 1:i1 + 1]
    t0 = rows[i0][2]
    print("# one step's kernel timeline ({} dispatches)\n".format(len(step)))
    print("| # | kernel | {} | dur us | gap us |".format(" | ".join(extra)))
    print("|---:|---|{}---:|---:|".format("---|" * len(extra)))
    busy = gaps = 0.0
    last_end = t0
    agg = {}
    for k, r in enumerate(step):
        name, s, e = r[0], r[1], r[2]
        dur = (e - s) / 1e3
        gap = max(0.0, (s - last_end) / 1e3)
        busy += dur
        gaps += gap
        last_end = max(last_end, e)
        sn = _short(name)
        c, t = agg.get(sn, (0, 0.0))
        agg[sn] = (c + 1, t + dur)
        print("| {} | {} | {} | {:.1f} | {:.1f} |".format(
            k, sn, " | ".join(str(x) for x in r[3:]), dur, gap))
    wall = (step[-1][2] - t0) / 1e3
    print("\nstep wall {:.1f} us = kernel time {:.1f} us (overlap counted once: {:.1f}) "
          "+ gaps {:.1f} us\n".format(wall, busy, wall - gaps, gaps))
    print("| kernel | calls | total us | avg us |\n|---|---:|---:|---:|")
    for sn, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print("| {} | {} | {:.1f} | {:.1f} |".format(sn, c, t, t / c))


if __name__ == "__main__":
    main()
