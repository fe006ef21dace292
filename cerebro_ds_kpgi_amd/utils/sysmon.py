"""1 Hz system telemetry sampler.

Replaces the reference's shell loggers (``logs/bin/{gpu,cpu,disk,network}
_logger.sh``: nvidia-smi, vmstat/free, iostat, sar) with one background
thread per node that samples

* GPU: utilisation, HBM used, power — ``amd-smi metric --json`` (falls back
  to ``rocm-smi --json``, then to ``torch.cuda`` memory counters),
* xGMI: per-link cumulative read / write KB between every GPU pair —
  ``amd-smi xgmi --metric --json`` (the model-hop data plane's links; absent
  on single-GPU boxes and when amd-smi cannot read them: the sample then
  has no ``xgmi`` key),
* CPU / memory: ``/proc/stat``, ``/proc/meminfo``,
* disk: ``/proc/diskstats`` (sectors read / written),
* network: ``/proc/net/dev`` (bytes rx / tx),

and appends one JSON object per sample to ``{dir}/sysmon_{host}.jsonl``.
``summarize`` reproduces ``SystemLogAnalyzer``'s report (mean utilisation, GB
read / written, GB over network; ``plots/data_analytics.py:200-477``) and
adds the GB moved over xGMI per GPU (the reference's per-node network
logger, ``logs/bin/network_logger.sh:12-19``, is what attributes hop cost
there).
"""

import json
import os
import shutil
import socket
import subprocess
import threading
import time


def _read(path):
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return ""


def cpu_times():
    line = _read("/proc/stat").splitlines()[0].split()
    vals = [int(v) for v in line[1:]]
    idle = vals[3] + (vals[4] if len(vals) > 4 else 0)
    return sum(vals), idle


def meminfo():
    out = {}
    for line in _read("/proc/meminfo").splitlines():
        k, _, v = line.partition(":")
        if k in ("MemTotal", "MemAvailable"):
            out[k] = int(v.split()[0]) * 1024
    return out


def disk_bytes():
    rd = wr = 0
    for line in _read("/proc/diskstats").splitlines():
        f = line.split()
        if len(f) > 9 and not f[2].startswith(("loop", "ram")):
            rd += int(f[5]) * 512
            wr += int(f[9]) * 512
    return rd, wr


def net_bytes():
    rx = tx = 0
    for line in _read("/proc/net/dev").splitlines()[2:]:
        name, _, rest = line.partition(":")
        if name.strip() == "lo":
            continue
        f = rest.split()
        if len(f) >= 9:
            rx += int(f[0])
            tx += int(f[8])
    return rx, tx


def gpu_metrics():
    """List of per-GPU dicts {util, mem_used, power} (best effort)."""
    if shutil.which("amd-smi"):
        try:
            r = subprocess.run(["amd-smi", "metric", "--usage", "--mem-usage", "--power",
                                "--json"], capture_output=True, text=True, timeout=10)
            data = json.loads(r.stdout) if r.returncode == 0 and r.stdout.strip() else None
            if isinstance(data, list):
                out = []
                for d in data:
                    u = d.get("usage", {}) or {}
                    m = d.get("mem_usage", {}) or {}
                    p = d.get("power", {}) or {}
                    out.append({"util": _num(u.get("gfx_activity")),
                                "mem_used": _num(m.get("used_vram")),
                                "power": _num(p.get("socket_power"))})
                return out
        except (OSError, ValueError, subprocess.SubprocessError):
            pass
    try:
        import torch
        if torch.cuda.is_available():
            return [{"util": None, "mem_used": torch.cuda.memory_allocated(i) / 2 ** 20,
                     "power": None} for i in range(torch.cuda.device_count())]
    except Exception:  # pragma: no cover
        pass
    return []


def parse_xgmi(data):
    """``amd-smi xgmi --metric --json`` output -> ``[{"gpu", "bit_rate",
    "links": [{"peer", "read_kb", "write_kb"}]}]``.  The CLI's JSON nests
    the per-GPU records differently across versions (a list, or a dict
    holding one); every dict carrying ``link_metrics`` is one GPU."""
    found = []

    def walk(o):
        if isinstance(o, dict):
            if "link_metrics" in o:
                found.append(o)
                return
            for v in o.values():
                walk(v)
        elif isinstance(o, list):
            for v in o:
                walk(v)
    walk(data)
    out = []
    for g in found:
        lm = g.get("link_metrics") or {}
        links = []
        for ln in lm.get("links") or []:
            rd, wr = _num(ln.get("read")), _num(ln.get("write"))
            if rd is None and wr is None:
                continue                     # "N/A": no link to that GPU (itself)
            links.append({"peer": ln.get("gpu"), "read_kb": rd, "write_kb": wr})
        out.append({"gpu": g.get("gpu"), "bit_rate": _num(lm.get("bit_rate")), "links": links})
    return out


def xgmi_metrics():
    """Per-GPU xGMI link counters (``parse_xgmi``), or [] when unavailable."""
    if not shutil.which("amd-smi"):
        return []
    try:
        r = subprocess.run(["amd-smi", "xgmi", "--metric", "--json"], capture_output=True,
                           text=True, timeout=10)
        if r.returncode != 0 or not r.stdout.strip():
            return []
        return [g for g in parse_xgmi(json.loads(r.stdout)) if g["links"]]
    except (OSError, ValueError, subprocess.SubprocessError):
        return []


def _num(v):
    if isinstance(v, dict):
        v = v.get("value")
    try:
        return float(v)
    except (TypeError, ValueError):
        return None


class SysMonitor(object):
    def __init__(self, directory, interval=1.0, gpus=True, xgmi=True):
        self.dir = directory
        self.interval = interval
        self.gpus = gpus
        self.xgmi = xgmi
        self.path = os.path.join(directory, "sysmon_{}.jsonl".format(socket.gethostname()))
        self._stop = threading.Event()
        self._t = None

    def sample(self, prev):
        tot, idle = cpu_times()
        d = {"ts": time.time(), "cpu_total": tot, "cpu_idle": idle}
        d.update(meminfo())
        d["disk_read"], d["disk_write"] = disk_bytes()
        d["net_rx"], d["net_tx"] = net_bytes()
        if self.gpus:
            d["gpus"] = gpu_metrics()
        if self.xgmi:
            x = xgmi_metrics()
            if x:
                d["xgmi"] = x
            else:
                self.xgmi = False            # not on this box: stop asking
        if prev:
            dt = max(tot - prev["cpu_total"], 1)
            d["cpu_util"] = 100.0 * (1 - (idle - prev["cpu_idle"]) / dt)
        return d

    def _run(self):
        os.makedirs(self.dir, exist_ok=True)
        prev = None
        with open(self.path, "a") as f:
            while not self._stop.is_set():
                prev = self.sample(prev)
                f.write(json.dumps(prev) + "\n")
                f.flush()
                self._stop.wait(self.interval)

    def start(self):
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()
        return self

    def stop(self):
        self._stop.set()
        if self._t:
            self._t.join(timeout=5)


def summarize(path):
    rows = [json.loads(l) for l in open(path) if l.strip()]
    if not rows:
        return {}
    a, b = rows[0], rows[-1]
    cpu = [r["cpu_util"] for r in rows if "cpu_util" in r]
    gutil = [g["util"] for r in rows for g in r.get("gpus", []) if g.get("util") is not None]
    out = {"seconds": b["ts"] - a["ts"],
           "cpu_util_mean": sum(cpu) / len(cpu) if cpu else None,
           "gpu_util_mean": sum(gutil) / len(gutil) if gutil else None,
           "disk_read_gb": (b["disk_read"] - a["disk_read"]) / 1e9,
           "disk_write_gb": (b["disk_write"] - a["disk_write"]) / 1e9,
           "net_gb": ((b["net_rx"] - a["net_rx"]) + (b["net_tx"] - a["net_tx"])) / 1e9}
    xr = [r for r in rows if r.get("xgmi")]
    if len(xr) >= 2:
        out["xgmi_write_gb"] = _xgmi_delta(xr[0]["xgmi"], xr[-1]["xgmi"], "write_kb")
        out["xgmi_read_gb"] = _xgmi_delta(xr[0]["xgmi"], xr[-1]["xgmi"], "read_kb")
    return out


def _xgmi_delta(first, last, field):
    """{gpu: GB} of ``field`` moved between two samples, over all its links."""
    def table(sample):
        return {(g["gpu"], ln["peer"]): ln.get(field) for g in sample for ln in g["links"]}
    t0, t1 = table(first), table(last)
    out = {}
    for (gpu, peer), v1 in t1.items():
        v0 = t0.get((gpu, peer))
        if v0 is None or v1 is None:
            continue
        out[str(gpu)] = out.get(str(gpu), 0.0) + max(0.0, v1 - v0) / 1e6
    return out
