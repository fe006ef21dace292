"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE and
WRITE_SIZE, one pass each: ``scripts/gpu/hbm_pmc.sh``).

Prints, per kernel (template arguments folded), the dispatches, MB read and
written per training step (normalised by the Adam dispatches: one per step),
kernel time per step under the counter pass and the achieved HBM GB/s —
the bytes half of the roofline that ``tools.roofline`` prices analytically.

    python -m cerebro_ds_kpgi_amd.tools.hbm_pmc gpurun_out/hbm_c8 [--top 30]
    python -m cerebro_ds_kpgi_amd.tools.hbm_pmc gpurun_out/hbm_c8 --dispatches [--hbm 6.0]

``--dispatches`` lists the last step's dispatches one by one (grid size
identifies the layer) ranked by their gap to the HBM floor: time minus
(read + written bytes) / ``--hbm`` TB/s.
"""

import argparse
import collections
import csv
import os
import re

from .prof_summary import family


def short(name):
    n = re.sub(r"\(.*", "", name)
    n = re.sub(r"^void ", "", n)
    return n[:70]


def read_pass(d, ctr, last_steps):
    """{kernel: [calls, KB, ns]} over the dispatches of the last
    ``last_steps`` training steps (step boundary = the Adam dispatch)."""
    path = os.path.join(d, ctr, "p_counter_collection.csv")
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Dispatch_Id"]))
    adam = [int(r["Dispatch_Id"]) for r in rows if "adam_kernel" in r["Kernel_Name"]]
    lo, hi = -1, float("inf")
    if last_steps and len(adam) > last_steps:
        lo, hi = adam[-last_steps - 1], adam[-1]
    out = collections.defaultdict(lambda: [0, 0.0, 0.0])     # calls, KB, ns
    for r in rows:
        if not lo < int(r["Dispatch_Id"]) <= hi:
            continue
        k = short(r["Kernel_Name"])
        o = out[k]
        o[0] += 1
        o[1] += float(r["Counter_Value"])
        o[2] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    return out


def read_dispatches(d, ctr):
    """The last training step's dispatches (between the last two Adam
    dispatches): [(dispatch id, kernel, grid, ns, bytes)]."""
    path = os.path.join(d, ctr, "p_counter_collection.csv")
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Dispatch_Id"]))
    adam = [int(r["Dispatch_Id"]) for r in rows if "adam_kernel" in r["Kernel_Name"]]
    lo, hi = (adam[-2], adam[-1]) if len(adam) >= 2 else (-1, float("inf"))
    out = []
    for r in rows:
        i = int(r["Dispatch_Id"])
        if lo < i <= hi:
            out.append((i, short(r["Kernel_Name"]), int(r.get("Grid_Size", 0) or 0),
                        float(r["End_Timestamp"]) - float(r["Start_Timestamp"]),
                        float(r["Counter_Value"]) * 1e3))
    return out


def dispatch_table(d, top, hbm_tbs):
    fe = read_dispatches(d, "FETCH_SIZE")
    wr = {i: b for i, _, _, _, b in read_dispatches(d, "WRITE_SIZE")}
    rows = []
    for i, k, grid, ns, rb in fe:
        wb = wr.get(i, 0.0)
        floor_ns = (rb + wb) / (hbm_tbs * 1e12) * 1e9
        rows.append((ns - floor_ns, i, k, grid, ns, rb, wb, floor_ns))
    rows.sort(reverse=True)
    tot = sum(r[4] for r in rows)
    gap = sum(max(r[0], 0.0) for r in rows)
    print("# last step: {} dispatches, {:.0f} us of kernel time, {:.0f} us above the HBM floor "
          "at {} TB/s".format(len(rows), tot / 1e3, gap / 1e3, hbm_tbs))
    print()
    print("| dispatch | kernel | grid | us | MB read | MB written | floor us | gap us |")
    print("|---:|---|---:|---:|---:|---:|---:|---:|")
    for g, i, k, grid, ns, rb, wb, fl in rows[:top]:
        print("| {} | `{}` | {} | {:.1f} | {:.1f} | {:.1f} | {:.1f} | {:.1f} |".format(
            i, k, grid, ns / 1e3, rb / 1e6, wb / 1e6, fl / 1e3, g / 1e3))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--last-steps", type=int, default=2)
    ap.add_argument("--dispatches", action="store_true")
    ap.add_argument("--hbm", type=float, default=6.0, help="HBM roof in TB/s")
    a = ap.parse_args(argv)
    if a.dispatches:
        dispatch_table(a.dir, a.top, a.hbm)
        return
    fe = read_pass(a.dir, "FETCH_SIZE", a.last_steps)
    wr = read_pass(a.dir, "WRITE_SIZE", a.last_steps)
    steps = sum(v[0] for k, v in fe.items() if k.startswith("adam_kernel")) or 1
    rows = []
    for k in set(fe) | set(wr):
        c, rk, t = fe.get(k, [0, 0.0, 0.0])
        _, wk, t2 = wr.get(k, [0, 0.0, 0.0])
        ns = max(t, t2)
        rows.append((k, c / steps, rk / 1e3 / steps, wk / 1e3 / steps, ns / 1e3 / steps))
    rows.sort(key=lambda r: -(r[2] + r[3]))
    tot_r = sum(r[2] for r in rows)
    tot_w = sum(r[3] for r in rows)
    tot_us = sum(r[4] for r in rows)
    print("# HBM traffic per training step ({} steps in the pass; FETCH_SIZE / WRITE_SIZE)"
          .format(steps))
    print()
    print("total: {:.0f} MB read + {:.0f} MB written = {:.2f} GB per step; kernel time under "
          "the counter pass {:.2f} ms -> {:.0f} GB/s average".format(
              tot_r, tot_w, (tot_r + tot_w) / 1e3, tot_us / 1e3,
              (tot_r + tot_w) / 1e3 / max(tot_us / 1e6, 1e-12)))
    print()
    fam = collections.defaultdict(lambda: [0.0, 0.0, 0.0])
    for k, c, r, w, us in rows:
        f = fam[family(k)]
        f[0] += r
        f[1] += w
        f[2] += us
    print("| family | MB read | MB written | us | GB/s |")
    print("|---|---:|---:|---:|---:|")
    for k, (r, w, us) in sorted(fam.items(), key=lambda kv: -(kv[1][0] + kv[1][1])):
        print("| {} | {:.0f} | {:.0f} | {:.0f} | {:.0f} |".format(k, r, w, us,
                                                               (r + w) / max(us, 1e-9) * 1e3))
    print()
    print("| kernel | calls/step | MB read | MB written | us | GB/s |")
    print("|---|---:|---:|---:|---:|---:|")
    for k, c, r, w, us in rows[:a.top]:
        print("| `{}` | {:.1f} | {:.0f} | {:.0f} | {:.0f} | {:.0f} |".format(
            k, c, r, w, us, (r + w) / max(us, 1e-9) * 1e3))


if __name__ == "__main__":
    main()
