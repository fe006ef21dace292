"""Concurrency evidence from a rocprofv3 kernel trace: for every dispatch of
a kernel (name substring, optional grid filter), how much of its lifetime
other kernels were running beside it (union of their intervals).

    python -m cerebro_ds_kpgi_amd.tools.prof_overlap gpurun_out/prof_X/prof_results.db \\
        --kernel wgrad_batch32 --grid 24576 --last 10

Used for the side-stream wgrad batch (profiles/r2_ab_wgrad_chunk.md).
"""

import argparse
import glob
import os
import sqlite3


def _db(path):
    if os.path.isdir(path):
        found = sorted(glob.glob(os.path.join(path, "**", "*.db"), recursive=True))
        if not found:
            raise SystemExit("no .db under " + path)
        return found[0]
    return path


def overlap(db, kernel, grid=None, last=10):
    con = sqlite3.connect(_db(db))
    rows = con.execute("select name, start, end, grid_x from kernels order by start").fetchall()
    mine = [r for r in rows if kernel in r[0] and (grid is None or r[3] == grid)][-last:]
    out = []
    for name, s, e, _ in mine:
        iv = sorted((max(s, b), min(e, c)) for n, b, c, _ in rows
                    if b < e and c > s and kernel not in n)
        busy, cs, ce, count = 0, None, None, len(iv)
        for a, b in iv:
            if ce is None or a > ce:
                if ce is not None:
                    busy += ce - cs
                cs, ce = a, b
            else:
                ce = max(ce, b)
        if ce is not None:
            busy += ce - cs
        out.append({"ms": (e - s) / 1e6, "covered": busy / max(e - s, 1), "kernels": count})
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--grid", type=int, default=None, help="grid_x (threads) filter")
    ap.add_argument("--last", type=int, default=10)
    a = ap.parse_args(argv)
    res = overlap(a.db, a.kernel, a.grid, a.last)
    if not res:
        raise SystemExit("no matching dispatch")
    n = len(res)
    print("{} dispatches of '{}': mean {:.3f} ms, other kernels running during {:.1f} % of "
          "their time, {:.0f} overlapping dispatches each".format(
              n, a.kernel, sum(r["ms"] for r in res) / n,
              100 * sum(r["covered"] * r["ms"] for r in res) / sum(r["ms"] for r in res),
              sum(r["kernels"] for r in res) / n))


if __name__ == "__main__":
    main()
