"""Run-log analytics: makespan, time breakdown, learning curves, telemetry
(SURVEY.md §2.12 G8/G9, §5.1).

Reference: ``LogAnalyzer`` / ``SystemLogAnalyzer``
(``plots/data_analytics.py:168-190, 200-477, 719-1075``) and the
``semantics`` event->category tables of ``plots/plots.ipynb`` cell 0, which
map log intervals to {initialization, data_transmission, model_hopping,
train_valid, idle, exiting, merge}.  Here the same categories are computed
from this framework's own structured logs:

* ``global.log``  — ``{exp}, Start time:`` / ``End time:`` lines (makespan,
  parsed exactly like ``get_all_start_end``),
* ``jobs_info.pkl`` — one record per (config, partition) sub-epoch job with
  its rank, hop and train/valid wall times,
* ``summary.json`` — ETL (data load) seconds and final per-config curves,
* ``traces/trace_rank*.json`` — chrome-trace spans (checkpoint time),
* ``sys_logs/sysmon_*.jsonl`` — the 1 Hz telemetry sampler.

Per-rank busy time is split into model_hopping / train_valid / checkpoint;
``idle = makespan - initialization - busy`` for each rank (what the
reference attributes to stragglers and barriers).

    python -m cerebro_ds_kpgi_amd.tools.log_analyzer --logs_root LOGS [--exp NAME] [--json out]
"""

import argparse
import collections
import datetime
import glob
import json
import os

from ..utils import safe_pickle

TIME_FORMAT = "%Y-%m-%d %H:%M:%S"
CATEGORIES = ("initialization", "data_transmission", "model_hopping", "train_valid",
              "checkpoint", "idle")


def get_all_start_end(global_log, exp=None):
    """{exp: (start_dt, end_dt)} from ``global.log`` (last complete bracket)."""
    out = {}
    cur = {}
    with open(global_log) as f:
        for line in f:
            line = line.rstrip()
            name = line.split(",")[0]
            if exp is not None and name != exp:
                continue
            if "Start time" in line or "End time" in line:
                dt = datetime.datetime.strptime(" ".join(line.split(" ")[-2:]), TIME_FORMAT)
                if "Start time" in line:
                    cur[name] = dt
                elif name in cur:
                    out[name] = (cur.pop(name), dt)
    return out


def _load_jobs(logs_root):
    p = os.path.join(logs_root, "jobs_info.pkl")
    if os.path.exists(p):
        with open(p, "rb") as f:        # written by runtime.checkpoint.dump_infos
            return safe_pickle.load(f)
    p = os.path.join(logs_root, "jobs_info.json")
    if os.path.exists(p):
        with open(p) as f:
            return {int(e): d for e, d in json.load(f).items()}
    return {}


def breakdown(jobs_info, makespan, init_s=0.0, checkpoint_s=None, n_ranks=None):
    """Category seconds summed over ranks (GPU-seconds), plus per-epoch rows.

    A sub-epoch job runs on one rank; jobs of one round on the same rank ran
    packed in ONE launch, so their wall intervals are merged, not summed.
    """
    per_rank = collections.defaultdict(lambda: {"hop": [], "busy": []})
    per_epoch = {}
    for epoch, jobs in sorted(jobs_info.items()):
        e_start, e_end = float("inf"), 0.0
        for job in jobs.values():
            r = job.get("rank", 0)
            hop = (job["start_time"], job["start_time"] + job["hop_time"])
            busy = (hop[1], job["end_time"])
            per_rank[r]["hop"].append(hop)
            per_rank[r]["busy"].append(busy)
            e_start, e_end = min(e_start, job["start_time"]), max(e_end, job["end_time"])
        per_epoch[epoch] = {"seconds": e_end - e_start, "jobs": len(jobs)}
    ranks = n_ranks or max(len(per_rank), 1)
    tot = dict.fromkeys(CATEGORIES, 0.0)
    tot["initialization"] = init_s * ranks
    for r, iv in per_rank.items():
        tot["model_hopping"] += _union(iv["hop"])
        tot["train_valid"] += _union(iv["busy"])
    if checkpoint_s:
        tot["checkpoint"] = checkpoint_s
    busy = sum(tot[k] for k in CATEGORIES if k != "idle")
    tot["idle"] = max(makespan * ranks - busy, 0.0)
    frac = {k: v / max(makespan * ranks, 1e-9) for k, v in tot.items()}
    return {"gpu_seconds": tot, "fraction": frac, "per_epoch": per_epoch, "ranks": ranks}


def _union(intervals):
    total, end = 0.0, -float("inf")
    for a, b in sorted(intervals):
        if b <= end:
            continue
        total += b - max(a, end)
        end = b
    return total


def find_best(mst_state, top5=True):
    """Config with the lowest final valid error and its curve (``find_best``)."""
    key = "valid_top5_error" if top5 else "valid_top1_error"
    best, curve = None, None
    for m, st in mst_state.items():
        c = st.get(key) or []
        if c and (curve is None or c[-1] < curve[-1]):
            best, curve = m, c
    return best, list(range(1, len(curve or []) + 1)), curve or []


def trace_totals(logs_root):
    tot = collections.defaultdict(float)
    for p in glob.glob(os.path.join(logs_root, "traces", "trace_rank*.json")):
        with open(p) as f:
            for e in json.load(f)["traceEvents"]:
                if e.get("ph") == "X":
                    tot[e["name"]] += e["dur"] / 1e6
    return dict(tot)


def analyze(logs_root, exp=None):
    out = {"logs_root": logs_root}
    summ = {}
    sp = os.path.join(logs_root, "summary.json")
    if os.path.exists(sp):
        with open(sp) as f:
            summ = json.load(f)
    exp = exp or summ.get("approach")
    glog = os.path.join(os.path.dirname(os.path.abspath(logs_root)), "global.log")
    makespan = summ.get("makespan_s")
    if os.path.exists(glog):
        se = get_all_start_end(glog, exp)
        if se:
            name, (a, b) = sorted(se.items(), key=lambda kv: kv[1][1])[-1]
            out["exp"] = name
            out["start"], out["end"] = a.strftime(TIME_FORMAT), b.strftime(TIME_FORMAT)
            makespan = makespan or (b - a).total_seconds()
    jobs = _load_jobs(logs_root)
    tt = trace_totals(logs_root)
    if makespan is None and jobs:
        allj = [j for d in jobs.values() for j in d.values()]
        makespan = max(j["end_time"] for j in allj) - min(j["start_time"] for j in allj)
    out["makespan_s"] = makespan
    out["makespan_h"] = (makespan or 0) / 3600
    if jobs:
        out["breakdown"] = breakdown(jobs, makespan or 0.0, summ.get("etl_s", 0.0),
                                     tt.get("checkpoint"), summ.get("gpus"))
    if tt:
        out["trace_seconds"] = tt
    if summ.get("mst_state"):
        best, x, y = find_best(summ["mst_state"])
        out["best"] = {"model": best, "epochs": x, "valid_top5_error": y}
    sysf = glob.glob(os.path.join(logs_root, "sys_logs", "sysmon_*.jsonl"))
    if sysf:
        from ..utils.sysmon import summarize
        out["system"] = {os.path.basename(p): summarize(p) for p in sysf}
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--logs_root", required=True)
    ap.add_argument("--exp", default=None)
    ap.add_argument("--json", default="")
    a = ap.parse_args(argv)
    res = analyze(a.logs_root, a.exp)
    print("Method: {}".format(res.get("exp")))
    print("Total time: {} hrs".format(res["makespan_h"]))
    bd = res.get("breakdown")
    if bd:
        for k in CATEGORIES:
            print("  {:<18} {:10.1f} GPU-s  {:6.1%}".format(k, bd["gpu_seconds"][k],
                                                          bd["fraction"][k]))
    if "best" in res:
        print("Best config {}: valid top-5 error {}".format(res["best"]["model"],
                                                           res["best"]["valid_top5_error"]))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1, default=str)
    return res


if __name__ == "__main__":
    main()
