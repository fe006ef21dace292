"""Failure detection, requeue, resume and observability.

* a soft failure on one rank requeues only that rank's (config, partition)
  pairs; the run ends bit-identical to a fault-free run,
* a crash mid-epoch + ``resume=True`` from sub-epoch checkpoints ends
  bit-identical to an uninterrupted run (rotation and greedy schedulers),
* the heartbeat watchdog flags a silent rank,
* chrome-trace spans, per-job metrics JSONL and the system sampler.
"""

import json
import os
import time

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from test_distributed import _free_port, _msts


def _opts(outdir, **kw):
    from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions
    base = dict(n_train=64, n_valid=16, compute_dtype="fp32", verbose=False,
                models_root=os.path.join(outdir, "models"), logs_root=os.path.join(outdir, "logs"))
    base.update(kw)
    return EngineOptions(**base)


def _states(eng):
    return {m: eng.group_of[m].state_row(m).clone() for m in range(len(eng.msts))
            if eng.holder[m] in (None, eng.ctx.rank)}


def _run_soft(rank, world, port, outdir, fault):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                       "CEREBRO_BACKEND": "torch", "CEREBRO_QUIET": "1"})
    torch.set_num_threads(1)
    from cerebro_ds_kpgi_amd.parallel import init_distributed, shutdown
    from cerebro_ds_kpgi_amd.runtime.engine import MOPEngine
    ctx = init_distributed(device_type="cpu")
    eng = MOPEngine(_msts(), ctx, _opts(outdir, ckpt_every="none", fault_inject=fault))
    eng.run(2)
    torch.save(_states(eng), os.path.join(outdir, "states_{}.pt".format(rank)))
    if rank == 0:
        with open(os.path.join(outdir, "out.json"), "w") as f:
            json.dump({"failures": eng.failures, "images": eng.train_images,
                       "mst_state": {str(k): v for k, v in eng.mst_state.items()}}, f)
    eng.close()
    shutdown(ctx)


def _launch_soft(tmp, fault):
    os.makedirs(tmp, exist_ok=True)
    mp.spawn(_run_soft, args=(2, _free_port(), tmp, fault), nprocs=2, join=True)
    st = {}
    for r in range(2):
        st.update(torch.load(os.path.join(tmp, "states_{}.pt".format(r)), weights_only=True))
    with open(os.path.join(tmp, "out.json")) as f:
        return st, json.load(f)


def test_soft_fault_requeues_only_failed_pairs(tmp_path):
    ref, ref_out = _launch_soft(str(tmp_path / "ref"), "")
    got, out = _launch_soft(str(tmp_path / "flt"), "1:1:soft")
    fails = out["failures"]
    # rank 1 owns partitions 2 and 3 -> exactly those two pairs failed once
    assert sorted(f["partition"] for f in fails) == [2, 3]
    assert all(f["rank"] == 1 and f["subepoch"] == 1 and f["attempt"] == 0 for f in fails)
    assert out["mst_state"] == ref_out["mst_state"]
    assert set(got) == set(ref)
    for m in ref:
        assert torch.equal(got[m], ref[m]), m


def _engine(outdir, scheduler, **kw):
    from cerebro_ds_kpgi_amd.parallel import DistContext
    from cerebro_ds_kpgi_amd.runtime.engine import MOPEngine
    return MOPEngine(_msts(), DistContext(), _opts(outdir, scheduler=scheduler,
                                                   shuffle=True, **kw))


@pytest.mark.parametrize("scheduler", ["rotation", "greedy"])
def test_crash_then_resume_matches_uninterrupted(tmp_path, scheduler, monkeypatch):
    monkeypatch.setenv("CEREBRO_BACKEND", "torch")
    monkeypatch.setenv("CEREBRO_QUIET", "1")
    torch.set_num_threads(2)
    # sub-epoch checkpoints run the lock-step runtime; the reference run too
    # (the async runtime packs rows in another order: equal to float noise)
    ref = _engine(str(tmp_path / "ref"), scheduler, ckpt_every="none", runtime="lockstep")
    ref.run(2)
    want = _states(ref)
    ref.close()

    d = str(tmp_path / "run")
    eng = _engine(d, scheduler, ckpt_every="subepoch", fault_inject="0:6")   # epoch 2, round 3
    with pytest.raises(RuntimeError, match="FAULT INJECTED"):
        eng.run(2)
    eng.close()
    with open(os.path.join(d, "models", "resume.json")) as f:
        st = json.load(f)
    assert st["epoch"] == 2 and st["rounds_done"] == 2 and not st["epoch_done"]

    eng2 = _engine(d, scheduler, ckpt_every="subepoch", resume=True)
    eng2.run(2)
    got = _states(eng2)
    for m in want:
        assert torch.equal(got[m], want[m]), (scheduler, m)
    for m in range(len(ref.msts)):
        for k in ("train_loss", "valid_loss"):
            assert eng2.mst_state[m][k] == pytest.approx(ref.mst_state[m][k], rel=1e-6)
    eng2.close()


@pytest.mark.parametrize("crash_round", [1, 3])
def test_resume_more_configs_than_partitions(tmp_path, monkeypatch, crash_round):
    """S=4 configs on P=2 partitions: a crash in epoch 1 leaves configs that
    never trained (no committed checkpoint); resume starts them from their
    seeded initial state and ends bit-identical to an uninterrupted run."""
    monkeypatch.setenv("CEREBRO_BACKEND", "torch")
    monkeypatch.setenv("CEREBRO_QUIET", "1")
    torch.set_num_threads(2)
    ref = _engine(str(tmp_path / "ref"), "rotation", ckpt_every="none", runtime="lockstep",
                  slots_per_gpu=2)
    ref.run(1)
    want = _states(ref)
    ref.close()
    d = str(tmp_path / "run")
    eng = _engine(d, "rotation", ckpt_every="subepoch", slots_per_gpu=2,
                  fault_inject="0:{}".format(crash_round))
    with pytest.raises(RuntimeError, match="FAULT INJECTED"):
        eng.run(1)
    eng.close()
    with open(os.path.join(d, "models", "resume.json")) as f:
        st = json.load(f)
    assert st["rounds_done"] == crash_round
    if crash_round == 1:
        assert len(st["versions"]) == 2          # half the configs never trained
    eng2 = _engine(d, "rotation", ckpt_every="subepoch", slots_per_gpu=2, resume=True)
    eng2.run(1)
    got = _states(eng2)
    for m in want:
        assert torch.equal(got[m], want[m]), m
    eng2.close()


def test_interrupted_commit_keeps_previous_restart_point(tmp_path, monkeypatch):
    """Files of a commit that never published resume.json are ignored: the
    restart point stays the last complete commit, and publishing re-points
    the canonical CTQ files and deletes superseded versions."""
    from cerebro_ds_kpgi_amd.runtime.checkpoint import ckpt_path, read_checkpoint
    monkeypatch.setenv("CEREBRO_BACKEND", "torch")
    monkeypatch.setenv("CEREBRO_QUIET", "1")
    d = str(tmp_path)
    eng = _engine(d, "rotation", ckpt_every="epoch")
    eng.run(1)
    root = os.path.join(d, "models")
    p0 = ckpt_path(root, 0, eng.msts[0])
    w_committed = read_checkpoint(p0)[0].copy()
    assert os.path.exists(p0 + "@e1") and os.path.samefile(p0, p0 + "@e1")
    # a half-finished next commit: garbage weights under a newer version
    with open(p0 + "@e2", "wb") as f:
        f.write(np.full(w_committed.size, 7.0, "<f4").tobytes())
    eng.close()
    eng2 = _engine(d, "rotation", ckpt_every="epoch", resume=True)
    assert eng2._resume()[0] == 2
    grp = eng2.group_of[0]
    np.testing.assert_array_equal(grp.home.row_weights_f32(grp.home_row[0]), w_committed)
    eng2.run(2)
    assert not os.path.exists(p0 + "@e1")
    assert os.path.samefile(p0, p0 + "@e2") and os.path.exists(p0 + "@e2.json")
    assert not np.all(read_checkpoint(p0)[0] == 7.0)
    eng2.close()


def test_epoch_resume_skips_finished_epochs(tmp_path, monkeypatch):
    monkeypatch.setenv("CEREBRO_BACKEND", "torch")
    monkeypatch.setenv("CEREBRO_QUIET", "1")
    d = str(tmp_path)
    eng = _engine(d, "rotation", ckpt_every="epoch")
    eng.run(1)
    eng.close()
    eng2 = _engine(d, "rotation", ckpt_every="epoch", resume=True)
    eng2.run(2)
    assert eng2.round_idx == 8          # 4 rounds of epoch 1 restored + 4 run
    assert all(len(eng2.mst_state[m]["train_loss"]) == 2 for m in range(4))
    eng2.close()


def test_heartbeat_watchdog_flags_silent_rank(tmp_path):
    from torch.distributed import HashStore
    from cerebro_ds_kpgi_amd.parallel.health import Heartbeat
    store = HashStore()
    seen = []
    w0 = Heartbeat(store, 0, 2, interval=0.05, timeout=0.4, logs_root=str(tmp_path),
                   on_failure=seen.append)
    w1 = Heartbeat(store, 1, 2, interval=0.05, timeout=0.4)
    w1.start()
    w0.start()
    time.sleep(0.3)
    assert not seen and w0.check() == []
    w1.stop()                      # rank 1 goes silent
    deadline = time.time() + 5
    while not seen and time.time() < deadline:
        time.sleep(0.05)
    w0.stop()
    assert seen == [[1]]
    with open(os.path.join(str(tmp_path), "failed_workers.json")) as f:
        assert json.load(f)["lost"] == [1]


def test_watchdog_flags_rank_stalled_inside_a_job(tmp_path):
    """The beating thread keeps stamping while the training thread hangs:
    the progress record, not the stamp, reveals the stall; an idle rank is
    not flagged."""
    from cerebro_ds_kpgi_amd.parallel.health import Heartbeat
    store = torch.distributed.HashStore()
    seen = []
    w0 = Heartbeat(store, 0, 3, interval=0.05, timeout=5.0, logs_root=str(tmp_path),
                   on_failure=seen.append, stall_timeout=0.4)
    w1 = Heartbeat(store, 1, 3, interval=0.05, timeout=5.0)
    w2 = Heartbeat(store, 2, 3, interval=0.05, timeout=5.0)
    for w in (w1, w2, w0):
        w.start()
    w1.progress(3, busy=True)              # rank 1 enters a job and never leaves
    w2.progress(3, busy=False)             # rank 2 waits idle for work
    deadline = time.time() + 5
    while not seen and time.time() < deadline:
        w0.progress(int(time.time() * 100), busy=True)    # rank 0 keeps making progress
        time.sleep(0.05)
    for w in (w0, w1, w2):
        w.stop()
    assert seen == [[1]]
    with open(os.path.join(str(tmp_path), "failed_workers.json")) as f:
        assert json.load(f)["stalled"] == [1]


@pytest.mark.parametrize("runtime", ["lockstep", "async"])
def test_trace_spans_and_metrics_jsonl(tmp_path, monkeypatch, runtime):
    monkeypatch.setenv("CEREBRO_BACKEND", "torch")
    monkeypatch.setenv("CEREBRO_QUIET", "1")
    d = str(tmp_path)
    eng = _engine(d, "rotation", ckpt_every="none", trace=True, runtime=runtime)
    eng.run(1)
    eng.close()
    with open(os.path.join(d, "logs", "traces", "trace_rank0.json")) as f:
        ev = json.load(f)["traceEvents"]
    names = {e["name"] for e in ev}
    # lock-step: a hop phase per round; async: the exposed wait for arrivals
    assert {"hop" if runtime == "lockstep" else "wait_arrival", "train", "valid",
            "report"} <= names
    assert sum(e["name"] == "train" for e in ev) == 4
    with open(os.path.join(d, "logs", "metrics.jsonl")) as f:
        rows = [json.loads(l) for l in f]
    assert len(rows) == 16
    assert {r["partition"] for r in rows} == {0, 1, 2, 3}
    assert all(r["img_s"] > 0 and r["loss"] > 0 for r in rows)


def test_sysmon_sampler(tmp_path):
    from cerebro_ds_kpgi_amd.utils.sysmon import SysMonitor, summarize
    mon = SysMonitor(str(tmp_path), interval=0.05, gpus=False).start()
    time.sleep(0.3)
    mon.stop()
    s = summarize(mon.path)
    assert s["seconds"] > 0 and s["cpu_util_mean"] is not None
    assert s["disk_read_gb"] >= 0 and s["net_gb"] >= 0


def _xgmi_sample(kb):
    # the shape `amd-smi xgmi --metric --json` prints (amdsmi_commands.py
    # xgmi(): per source GPU a link_metrics dict, one link entry per GPU,
    # "N/A" for itself), for two GPUs
    return {"xgmi_metric": [
        {"gpu": g, "bdf": "0000:0{}:00.0".format(g),
         "link_metrics": {"bit_rate": {"value": 32, "unit": "Gb/s"},
                          "max_bandwidth": {"value": 512, "unit": "Gb/s"},
                          "link_type": "XGMI",
                          "links": [{"gpu": p, "bdf": "0000:0{}:00.0".format(p),
                                     "read": "N/A" if p == g else {"value": kb * (g + 1), "unit": "KB"},
                                     "write": "N/A" if p == g else {"value": 2 * kb * (g + 1), "unit": "KB"}}
                                    for p in range(2)]}}
        for g in range(2)]}


def test_sysmon_xgmi_schema(tmp_path):
    """xGMI link counters: parsed per GPU and link from
    the amd-smi JSON, written into the sysmon samples, and summarised as GB
    moved per GPU; a box without them (this one) leaves the key out."""
    from cerebro_ds_kpgi_amd.utils import sysmon
    x0 = sysmon.parse_xgmi(_xgmi_sample(1000))
    assert [g["gpu"] for g in x0] == [0, 1]
    assert x0[0]["bit_rate"] == 32
    assert x0[0]["links"] == [{"peer": 1, "read_kb": 1000.0, "write_kb": 2000.0}]
    x1 = sysmon.parse_xgmi(_xgmi_sample(1000 + 5e6))
    path = tmp_path / "sysmon_h.jsonl"
    base = {"cpu_total": 1, "cpu_idle": 0, "disk_read": 0, "disk_write": 0, "net_rx": 0,
            "net_tx": 0}
    with open(path, "w") as f:
        f.write(json.dumps(dict(base, ts=0.0, xgmi=x0)) + "\n")
        f.write(json.dumps(dict(base, ts=1.0, xgmi=x1)) + "\n")
    s = sysmon.summarize(str(path))
    assert s["xgmi_read_gb"] == {"0": pytest.approx(5.0), "1": pytest.approx(10.0)}
    assert s["xgmi_write_gb"] == {"0": pytest.approx(10.0), "1": pytest.approx(20.0)}
    mon = sysmon.SysMonitor(str(tmp_path), interval=0.05, gpus=False)
    d = mon.sample(None)
    assert "xgmi" not in d and mon.xgmi is False        # no GPUs here: not sampled again
