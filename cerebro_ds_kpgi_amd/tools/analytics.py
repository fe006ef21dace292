"""Cross-run analytics and figures (reference
``plots/data_analytics.py`` and ``plots/plots.ipynb``).

Reads both this framework's run logs and the reference's own log formats:

* reference run-log lines: ``parse_madlib_line`` (``info: timestamp (...)``),
  ``parse_ctq_line``, ``split_standalone_line`` / ``parse_standalone_line``
  (``EVENT: ..., TIME: <epoch s>``), ``parse_ctq_learning_curve`` (the dict
  printed before every ``ENDING BATCH:`` line), ``data_analytics.py:61-113``;
* job records: ``models_info`` ({model_key: [job dict]}, the CTQ
  ``model_info_ordered`` schema, which ``runtime.engine`` writes too) ->
  ``ctq_parse_model_info_ordered`` / ``ctq_find`` (best config's curve by
  validation metric or loss, ``data_analytics.py:115-158``);
* system telemetry: ``SystemLogs`` parses the reference's shell loggers
  (``logs/bin/{cpu,gpu,disk,network}_logger.sh``: a timestamp line, then a
  ``cpu%,mem%`` / nvidia-smi CSV / ``iostat -dm`` / two ``sar -n DEV`` lines)
  and this framework's ``sysmon_*.jsonl``, and reports what
  ``SystemLogAnalyzer`` reports (``data_analytics.py:200-477``): mean
  utilisation over workers, MB read / written per worker and in total, GB
  moved over the network, within the run's [start, end) window;
* figures (matplotlib, Agg): learning curves of the best config of every
  approach vs wall time and vs epoch (notebook cells 40-70), the runtime
  breakdown stacked bars (cells 74-108, categories of
  ``tools.log_analyzer.CATEGORIES``) and speed-up vs workers (the scalability
  study, cells 110-125).

    python -m cerebro_ds_kpgi_amd.tools.analytics --run ctq=LOGS1 --run udaf=LOGS2 \\
        --out report_dir [--scaling scaling.json]
"""

import argparse
import ast
import datetime
import glob
import json
import os

import numpy as np

from ..utils import safe_pickle

TIME_FORMAT = "%Y-%m-%d %H:%M:%S"


# ---------------------------------------------------------------------------
# reference log-line formats
# ---------------------------------------------------------------------------
def parse_madlib_line(line):
    _, info, timestamp = [x.strip() for x in line.split(": ")]
    timestamp = timestamp.split("(")[0].strip()
    return info, datetime.datetime.strptime(timestamp, TIME_FORMAT), timestamp


def parse_ctq_line(line, return_timestamp=False):
    parsed = [x.strip() for x in line.split(": ")]
    info, timestamp = parsed[:-1], parsed[-1]
    t = datetime.datetime.strptime(timestamp, TIME_FORMAT)
    return (info, t, timestamp) if return_timestamp else (info, t)


def split_standalone_line(line):
    kv = [x.split(": ") for x in line.strip().split(", ")]
    return dict(x for x in kv if len(x) == 2)


def parse_standalone_line(line):
    d = split_standalone_line(line)
    return d["EVENT"], datetime.datetime.fromtimestamp(int(d["TIME"])), d["TIME"]


def parse_ctq_learning_curve(lines):
    """Rows {batch, mst_key, validation_metrics}: the literal dict printed on
    the line before each ``ENDING BATCH:`` (``ast.literal_eval``: no code runs)."""
    rows = []
    batches = [ast.literal_eval(lines[i - 1]) for i, line in enumerate(lines)
               if "ENDING BATCH:" in line and i > 0]
    for b, batch in enumerate(batches):
        for key, val in batch.items():
            rows.append({"batch": b, "mst_key": key, "validation_metrics": val})
    return rows


# ---------------------------------------------------------------------------
# job records -> curves
# ---------------------------------------------------------------------------
def ctq_parse_model_info_ordered(models_info):
    """{model_key: [job dicts]} -> pandas DataFrame (one row per job)."""
    import pandas as pd
    rows = []
    for k, jobs in models_info.items():
        for j in jobs:
            r = dict(j)
            r["mst_str"] = k
            r.setdefault("model_key", k)
            rows.append(r)
    return pd.DataFrame(rows)


def ctq_find(df, mst_key=None, best=True, mode="metric"):
    """(epochs, curve, model_key) of the best config at the last epoch (or
    of ``mst_key``): ``mode='metric'`` -> 1 - mean validation top-5 metric,
    ``'loss'`` -> mean validation loss, per (epoch, model) over partitions."""
    agg = df.groupby(["epoch", "model_key"]).agg(
        {"loss_train": "mean", "metric_train": "mean", "loss_valid": "mean",
         "metric_valid": "mean"}).reset_index()
    col = "metric_valid" if mode == "metric" else "loss_valid"
    if best:
        last = agg[agg["epoch"] == agg["epoch"].max()].reset_index(drop=True)
        i = last[col].idxmax() if mode == "metric" else last[col].idxmin()
        mst_key = last.loc[i, "model_key"]
    sel = agg[agg["model_key"] == mst_key].sort_values("epoch")
    x = np.asarray(sel["epoch"])
    y = 1 - np.asarray(sel[col]) if mode == "metric" else np.asarray(sel[col])
    return x, y, mst_key


def load_models_info(logs_root):
    p = os.path.join(logs_root, "models_info.pkl")
    if os.path.exists(p):
        with open(p, "rb") as f:          # written by runtime.checkpoint.dump_infos
            return safe_pickle.load(f)
    return {}


def learning_curve(logs_root, mode="metric"):
    """Best config of one run: epochs, curve, the wall time at which each
    epoch of that config ended (seconds from the run's first job), key."""
    mi = load_models_info(logs_root)
    if not mi:
        return None
    df = ctq_parse_model_info_ordered(mi)
    x, y, key = ctq_find(df, mode=mode)
    t0 = df["start_time"].min()
    ends = df[df["model_key"] == key].groupby("epoch")["end_time"].max()
    t = np.asarray([ends[e] - t0 for e in x])
    return {"epochs": x.tolist(), "curve": y.tolist(), "time_s": t.tolist(), "model_key": key}


# ---------------------------------------------------------------------------
# system telemetry
# ---------------------------------------------------------------------------
def _readlines(path):
    with open(path) as f:
        return [l.rstrip("\n") for l in f if l.strip()]


def _ts(line):
    return datetime.datetime.strptime(line.strip(), TIME_FORMAT)


class SystemLogs(object):
    """SystemLogAnalyzer-equivalent over one directory of per-worker logs
    (reference file names ``{kind}_{worker}.log``; ``master`` is the
    coordinator and is excluded from worker means)."""

    def __init__(self, logs_root, start=None, end=None):
        self.logs_root = logs_root
        self.start = start or datetime.datetime.min
        self.end = end or datetime.datetime.max
        self.total_time = ((end - start).total_seconds()
                           if start is not None and end is not None else None)

    def _files(self, prefix):
        out = {}
        for p in sorted(glob.glob(os.path.join(self.logs_root, prefix + "*.log"))):
            worker = os.path.basename(p).split("_")[-1].split(".")[0]
            out[worker] = p
        return out

    def _records(self, path, nlines, parse):
        lines = _readlines(path)
        i, out = 0, []
        while i + nlines < len(lines) + 1:
            try:
                t = _ts(lines[i])
                val = parse(lines[i + 1:i + nlines])
                i += nlines
            except (ValueError, IndexError, KeyError):
                i += 1                       # torn / garbled sample: skip a line
                continue
            if self.start <= t < self.end:
                out.append((t, val))
        return out

    # per-kind sample parsers
    @staticmethod
    def _cpu(ls):
        cpu, mem = ls[0].split(",")[:2]
        return float(cpu.strip().rstrip("%")), float(mem.strip().rstrip("%"))

    @staticmethod
    def _gpu(ls):
        # nvidia-smi csv: "util %, mem util %, power W" (one line per GPU is
        # summarised by the first GPU, as the reference does)
        f = [x.strip() for x in ls[0].split(",")]
        return float(f[0].split()[0]), float(f[1].split()[0])

    @staticmethod
    def _disk(ls):
        toks = ls[0].split()
        pos = toks.index("MB_wrtn") + 1
        toks = toks[pos:]
        devs = []
        for j in range(0, len(toks) - 5, 6):
            d = toks[j:j + 6]
            devs.append({"Device": d[0], "tps": float(d[1]), "MB_read/s": float(d[2]),
                         "MB_wrtn/s": float(d[3]), "MB_read": float(d[4]),
                         "MB_wrtn": float(d[5])})
        if not devs:
            raise ValueError("no device")
        return devs

    @staticmethod
    def _net(ls):
        out = []
        for line in ls[:2]:
            kv = dict(x.split(": ") for x in line.split(", ") if ": " in x)
            out.append({k: float(v) for k, v in kv.items() if not k.endswith("IFACE")})
        return out

    def report_utilization(self, kind="cpu"):
        """Mean utilisation (%) over workers: kind cpu | memory | gpu | gpu_memory."""
        prefix, parse, idx = {"cpu": ("cpu_utilization_", self._cpu, 0),
                              "memory": ("cpu_utilization_", self._cpu, 1),
                              "gpu": ("gpu_utilization_", self._gpu, 0),
                              "gpu_memory": ("gpu_utilization_", self._gpu, 1)}[kind]
        per = []
        for w, p in self._files(prefix).items():
            if w == "master":
                continue
            rec = self._records(p, 2, parse)
            if rec:
                per.append(float(np.mean([v[idx] for _, v in rec])))
        return float(np.mean(per)) if per else None

    def report_disk(self):
        """{worker: {MB_i, MB_o}} (counter max - min per device, summed) + mean / sum."""
        per = {}
        for w, p in self._files("disk_").items():
            if w == "master":
                continue
            rec = self._records(p, 2, self._disk)
            by_dev = {}
            for _, devs in rec:
                for d in devs:
                    lo_hi = by_dev.setdefault(d["Device"], [[np.inf, -np.inf], [np.inf, -np.inf]])
                    for k, c in ((0, "MB_read"), (1, "MB_wrtn")):
                        lo_hi[k][0] = min(lo_hi[k][0], d[c])
                        lo_hi[k][1] = max(lo_hi[k][1], d[c])
            mi = sum(v[0][1] - v[0][0] for v in by_dev.values())
            mo = sum(v[1][1] - v[1][0] for v in by_dev.values())
            per[w] = {"MB_i": mi, "MB_o": mo, "MB_io": mi + mo}
        io = [v["MB_io"] for v in per.values()]
        return {"per_worker": per, "mean_io_MB": float(np.mean(io)) if io else 0.0,
                "sum_io_MB": float(np.sum(io)) if io else 0.0}

    def report_network(self):
        """Mean rx/tx kB/s per interface (control, experiment) for the master
        and the workers, and the total GB received over the experiment
        interface = (master + mean worker x workers) x run seconds."""
        stats = {}
        for w, p in self._files("network_").items():
            rec = self._records(p, 3, self._net)
            if not rec:
                continue
            stats[w] = {
                "control_rxkBs": float(np.mean([v[0].get("rxkB/s", 0.0) for _, v in rec])),
                "exp_rxkBs": float(np.mean([v[1].get("rxkB/s", 0.0) for _, v in rec])),
                "exp_txkBs": float(np.mean([v[1].get("txkB/s", 0.0) for _, v in rec])),
            }
        workers = [v for k, v in stats.items() if k != "master"]
        avg = (stats.get("master", {}).get("exp_rxkBs", 0.0) +
               (np.mean([v["exp_rxkBs"] for v in workers]) * len(workers) if workers else 0.0))
        total_gb = avg * (self.total_time or 0.0) / 1024 / 1024
        return {"per_host": stats, "avg_exp_rx_kBs": float(avg), "total_GB": float(total_gb)}


def sysmon_report(logs_root):
    """The same report over this framework's ``sys_logs/sysmon_*.jsonl``."""
    from ..utils.sysmon import summarize
    return {os.path.basename(p): summarize(p)
            for p in glob.glob(os.path.join(logs_root, "sys_logs", "sysmon_*.jsonl"))}


# ---------------------------------------------------------------------------
# figures
# ---------------------------------------------------------------------------
def _plt():
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    return plt


def plot_learning_curves(curves, path, x="time_s"):
    """curves: {approach: learning_curve() dict}; x = time_s | epochs."""
    plt = _plt()
    fig, ax = plt.subplots(figsize=(5, 4))
    for name, c in sorted(curves.items()):
        if c:
            xs = np.asarray(c[x]) / (3600.0 if x == "time_s" else 1.0)
            ax.plot(xs, c["curve"], marker="o", label=name)
    ax.set_xlabel("time (h)" if x == "time_s" else "epoch")
    ax.set_ylabel("best config validation top-5 error")
    ax.legend()
    fig.tight_layout()
    fig.savefig(path)
    plt.close(fig)
    return path


def plot_breakdown(breakdowns, path):
    """breakdowns: {approach: log_analyzer.breakdown()['fraction']} -> stacked bars."""
    from .log_analyzer import CATEGORIES
    plt = _plt()
    names = sorted(breakdowns)
    fig, ax = plt.subplots(figsize=(1.2 * len(names) + 2, 4))
    bottom = np.zeros(len(names))
    for cat in CATEGORIES:
        vals = np.asarray([breakdowns[n].get(cat, 0.0) for n in names])
        ax.bar(names, vals, bottom=bottom, label=cat)
        bottom += vals
    ax.set_ylabel("fraction of GPU time")
    ax.legend(fontsize=7)
    fig.tight_layout()
    fig.savefig(path)
    plt.close(fig)
    return path


def plot_scaling(points, path):
    """points: {approach: {workers: makespan_s}} -> speed-up vs workers."""
    plt = _plt()
    fig, ax = plt.subplots(figsize=(5, 4))
    top = 1
    for name, pts in sorted(points.items()):
        ws = sorted(int(w) for w in pts)
        base = pts[str(ws[0])] if str(ws[0]) in pts else pts[ws[0]]
        sp = [base / (pts[str(w)] if str(w) in pts else pts[w]) * ws[0] for w in ws]
        ax.plot(ws, sp, marker="o", label=name)
        top = max(top, ws[-1])
    ax.plot([1, top], [1, top], "k--", lw=0.8, label="linear")
    ax.set_xlabel("workers (GPUs)")
    ax.set_ylabel("speed-up")
    ax.legend()
    fig.tight_layout()
    fig.savefig(path)
    plt.close(fig)
    return path


def report(runs, out_dir, scaling=None):
    """runs: {approach: logs_root}.  Writes report.json + figures."""
    from .log_analyzer import analyze
    os.makedirs(out_dir, exist_ok=True)
    res = {"runs": {}}
    curves, bds = {}, {}
    for name, root in runs.items():
        a = analyze(root, None)
        r = {"makespan_s": a.get("makespan_s")}
        lc = learning_curve(root)
        if lc:
            curves[name] = lc
            r["best"] = {"model_key": lc["model_key"], "final_error": lc["curve"][-1]}
        if "breakdown" in a:
            bds[name] = a["breakdown"]["fraction"]
            r["breakdown"] = a["breakdown"]["fraction"]
        sysm = sysmon_report(root)
        if sysm:
            r["system"] = sysm
        res["runs"][name] = r
    figs = []
    if curves:
        figs.append(plot_learning_curves(curves, os.path.join(out_dir, "learning_curves_time.png")))
        figs.append(plot_learning_curves(curves, os.path.join(out_dir, "learning_curves_epoch.png"),
                                         x="epochs"))
    if bds:
        figs.append(plot_breakdown(bds, os.path.join(out_dir, "breakdown.png")))
    if scaling:
        figs.append(plot_scaling(scaling, os.path.join(out_dir, "scaling.png")))
        res["scaling"] = scaling
    res["figures"] = [os.path.basename(f) for f in figs]
    res["curves"] = curves
    with open(os.path.join(out_dir, "report.json"), "w") as f:
        json.dump(res, f, indent=1, default=str)
    return res


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--run", action="append", default=[], help="approach=logs_root")
    ap.add_argument("--out", required=True)
    ap.add_argument("--scaling", default="", help="JSON {approach: {workers: makespan_s}}")
    a = ap.parse_args(argv)
    runs = dict(r.split("=", 1) for r in a.run)
    sc = None
    if a.scaling:
        with open(a.scaling) as f:
            sc = json.load(f)
    res = report(runs, a.out, sc)
    print(json.dumps({k: v for k, v in res.items() if k != "curves"}, indent=1, default=str))
    return res


if __name__ == "__main__":
    main()
