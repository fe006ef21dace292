"""Analytics parity: the reference's log formats (run-log lines, shell
system loggers) and SystemLogAnalyzer-style reports, best-config learning
curves from job records, and the report figures."""

import datetime
import os

import pytest

from cerebro_ds_kpgi_amd.tools import analytics as A


def _w(path, lines):
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def test_reference_line_parsers():
    info, t, _ = A.parse_standalone_line("EVENT: TRAIN_START, MST: 3, TIME: 1600000000")
    assert info == "TRAIN_START" and t == datetime.datetime.fromtimestamp(1600000000)
    info, t = A.parse_ctq_line("SUBEPOCH: 2: 2020-01-02 03:04:05")
    assert info == ["SUBEPOCH", "2"] and t.hour == 3
    info, t, _ = A.parse_madlib_line("x: EPOCH 1: 2020-01-02 03:04:05 (12.3s)")
    assert info == "EPOCH 1" and t.second == 5
    rows = A.parse_ctq_learning_curve(["{'a': 0.5, 'b': 0.7}", "ENDING BATCH:0, FINISHED:2",
                                       "{'c': 0.4}", "ENDING BATCH:1, FINISHED:3"])
    assert [(r["batch"], r["mst_key"]) for r in rows] == [(0, "a"), (0, "b"), (1, "c")]


def test_reference_system_logs(tmp_path):
    d = str(tmp_path)
    t0 = "2020-01-01 00:00:0{}"
    for w, cpu in (("worker0", 50), ("worker1", 70), ("master", 5)):
        _w(os.path.join(d, "cpu_utilization_{}.log".format(w)),
           [t0.format(0), "{}%,40.0%".format(cpu), t0.format(1), "{}%,60.0%".format(cpu + 10)])
        _w(os.path.join(d, "gpu_utilization_{}.log".format(w)),
           [t0.format(0), "90 %, 30 %, 250.00 W", t0.format(1), "garbled", t0.format(2),
            "70 %, 10 %, 200.00 W"])
        hdr = "Device tps MB_read/s MB_wrtn/s MB_read MB_wrtn"
        _w(os.path.join(d, "disk_{}.log".format(w)),
           [t0.format(0), hdr + " sda 1.0 0.1 0.2 100 200 sdb 1.0 0.1 0.2 10 20",
            t0.format(1), hdr + " sda 1.0 0.1 0.2 160 230 sdb 1.0 0.1 0.2 10 25"])
        net = ("{}_IFACE: eth{}, rxpck/s: 1.0, txpck/s: 1.0, rxkB/s: {}, txkB/s: 2.0, "
               "rxcmp/s: 0.0, txcmp/s: 0.0, rxmcst/s: 0.0, %ifutil: 0.1")
        _w(os.path.join(d, "network_{}.log".format(w)),
           [t0.format(0), net.format("CONTROL", 0, 1.0), net.format("EXPERIMENT", 1, 1024.0),
            t0.format(1), net.format("CONTROL", 0, 3.0), net.format("EXPERIMENT", 1, 3072.0)])
    start = datetime.datetime(2020, 1, 1)
    s = A.SystemLogs(d, start, start + datetime.timedelta(seconds=10))
    assert s.report_utilization("cpu") == pytest.approx((55 + 75) / 2)       # master excluded
    assert s.report_utilization("memory") == pytest.approx(50.0)
    assert s.report_utilization("gpu") == pytest.approx(80.0)                 # garbled skipped
    disk = s.report_disk()
    assert disk["per_worker"]["worker0"] == {"MB_i": 60.0, "MB_o": 35.0, "MB_io": 95.0}
    assert disk["sum_io_MB"] == pytest.approx(190.0)
    net = s.report_network()
    assert net["per_host"]["worker1"]["exp_rxkBs"] == pytest.approx(2048.0)
    # (master 2048 + mean worker 2048 x 2 workers) kB/s x 10 s
    assert net["total_GB"] == pytest.approx(3 * 2048.0 * 10 / 1024 / 1024)
    # a window that excludes the second sample
    s1 = A.SystemLogs(d, start, start + datetime.timedelta(seconds=1))
    assert s1.report_utilization("cpu") == pytest.approx(60.0)


def test_learning_curves_and_figures(tmp_path, monkeypatch):
    monkeypatch.setenv("CEREBRO_BACKEND", "torch")
    monkeypatch.setenv("CEREBRO_QUIET", "1")
    from cerebro_ds_kpgi_amd.parallel import DistContext
    from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine
    msts = [{"model": "tinycnn", "batch_size": 8, "learning_rate": lr, "lambda_value": 1e-4}
            for lr in (1e-3, 1e-2)]
    runs = {}
    for name, sched in (("ctq", "greedy"), ("udaf", "rotation")):
        root = str(tmp_path / name / "logs")
        eng = MOPEngine(msts, DistContext(), EngineOptions(
            scheduler=sched, n_train=32, n_valid=16, compute_dtype="fp32", verbose=False,
            ckpt_every="none", logs_root=root, slots_per_gpu=2))
        eng.run(2)
        eng.close()
        runs[name] = root
    res = A.report(runs, str(tmp_path / "rep"), scaling={"ctq": {"1": 100.0, "2": 55.0}})
    for f in ("learning_curves_time.png", "learning_curves_epoch.png", "breakdown.png",
              "scaling.png"):
        assert os.path.getsize(str(tmp_path / "rep" / f)) > 1000
    c = res["curves"]["ctq"]
    assert c["epochs"] == [1, 2] and len(c["curve"]) == 2 and c["time_s"][1] > c["time_s"][0]
    assert set(res["runs"]) == {"ctq", "udaf"}
