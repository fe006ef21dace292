"""Asynchronous MOP runtime (runtime/async_mop.py) on CPU with gloo.

* greedy on the event-driven runtime is work conserving: with injected
  heterogeneous job lengths its epoch makespan matches the greedy simulator
  (reference ``hetero_simluator.ipynb`` / scheduler.simulator) and beats the
  lock-step rotation that the reference's UDAF path runs,
* hops run on their own thread / stream / process group and overlap the
  receiver's validation: with a forced slow link the exposed hop time stays
  under 1 % of the run, where the lock-step runtime exposes every transfer,
* every (config, partition) pair runs exactly once per epoch; a job that
  stays on its GPU is a row re-assignment, not a state copy.
"""

import collections
import json
import os
import random
import statistics
import time

import pytest
import torch
import torch.multiprocessing as mp

from test_distributed import _free_port


def _cfgs(n):
    from cerebro_ds_kpgi_amd.config import catalog as cat
    from cerebro_ds_kpgi_amd.selection import get_msts
    base = get_msts(cat.param_grid_tiny)[0]
    out = []
    for i in range(n):
        m = dict(base)
        m["learning_rate"] = 1e-3 * (1 + i)
        out.append(m)
    return out


def _env(rank, world, port):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                       "CEREBRO_BACKEND": "torch", "CEREBRO_QUIET": "1"})
    torch.set_num_threads(1)


def _engine(ctx, S, slots, **kw):
    from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine
    base = dict(n_train=16, n_valid=8, compute_dtype="fp32", slots_per_gpu=slots,
                verbose=False, ckpt_every="none")
    base.update(kw)
    return MOPEngine(_cfgs(S), ctx, EngineOptions(**base))


def _pairs_once(eng, S, P):
    for e, jobs in eng.jobs_info.items():
        keys = sorted(jobs)
        assert len(keys) == S * P == len(set(keys)), (e, len(keys))


# ---------------------------------------------------------------------------
RUNTIMES = [0.15, 0.15, 0.15, 0.15, 0.45, 0.45, 0.75, 0.75]   # seconds per job of config m


def _makespan_worker(rank, world, port, outdir):
    _env(rank, world, port)
    from cerebro_ds_kpgi_amd.parallel import init_distributed, shutdown
    ctx = init_distributed(device_type="cpu")
    out = {}
    S = len(RUNTIMES)
    for name, sched, runtime in (("greedy_async", "greedy", "async"),
                                 ("rotation_lockstep", "rotation", "lockstep"),
                                 ("rotation_async", "rotation", "async")):
        eng = _engine(ctx, S, 1, scheduler=sched, runtime=runtime, sim_job_seconds=RUNTIMES)
        ctx.barrier()
        t0 = time.time()
        eng.run(1)
        out[name] = time.time() - t0
        _pairs_once(eng, S, world)
        eng.close()
    if rank == 0:
        with open(os.path.join(outdir, "makespan.json"), "w") as f:
            json.dump(out, f)
    shutdown(ctx)


def test_async_greedy_makespan_matches_simulator(tmp_path):
    from cerebro_ds_kpgi_amd.scheduler.simulator import simulate_greedy, simulate_rotation
    world = 3
    mp.spawn(_makespan_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
             join=True)
    with open(tmp_path / "makespan.json") as f:
        got = json.load(f)
    sims = sorted(simulate_greedy(RUNTIMES, world, rng=random.Random(s)) for s in range(200))
    sim_g = statistics.mean(sims)
    sim_g95 = sims[int(0.95 * len(sims))]         # the measured run is ONE draw of the policy
    sim_r = simulate_rotation(RUNTIMES, world)
    print("measured", got, "simulated greedy", sim_g, "rotation", sim_r)
    # work conserving: within 10 % of the event simulation of the same policy
    # (its 95th percentile: random tie-breaks make the makespan a distribution).
    # A loaded host (pytest -n) stretches every sleep-based job alike; the
    # lock-step rotation run measures that stretch, so scale the bound by it
    slow = max(1.0, got["rotation_lockstep"] / sim_r)
    assert got["greedy_async"] <= 1.10 * sim_g95 * slow, (sim_g, sim_g95)
    # and faster than lock-step rotation (simulated and measured)
    assert got["greedy_async"] < got["rotation_lockstep"]
    assert got["rotation_lockstep"] >= 0.95 * sim_r
    # data-flow rotation never loses to its lock-step execution
    assert got["rotation_async"] <= got["rotation_lockstep"] * 1.05


# ---------------------------------------------------------------------------
def _overlap_worker(rank, world, port, outdir):
    _env(rank, world, port)
    from cerebro_ds_kpgi_amd.parallel import init_distributed, shutdown
    ctx = init_distributed(device_type="cpu")
    out = {}
    for runtime in ("async", "lockstep"):
        eng = _engine(ctx, 2, 1, scheduler="rotation", runtime=runtime, trace=True,
                      hop_check=True, sim_job_seconds=[0.3], sim_valid_seconds=0.2,
                      sim_hop_seconds=0.1)
        ctx.barrier()
        t0 = time.time()
        eng.run(2)
        wall = time.time() - t0
        ev = [e for e in eng.tracer.events if e.get("ph") == "X"]
        hops = [(e["ts"], e["ts"] + e["dur"]) for e in ev if e["name"] == "hop"]
        valid = [(e["ts"], e["ts"] + e["dur"]) for e in ev if e["name"] == "valid"]
        overlap = sum(max(0.0, min(a1, b1) - max(a0, b0)) for a0, a1 in hops
                      for b0, b1 in valid) / 1e6
        out[runtime] = {"wall": wall, "exposed": eng.hop_time, "busy": eng.hop_busy_time,
                        "bytes": eng.hop_bytes, "overlap": overlap, "nhops": len(hops)}
        _pairs_once(eng, 2, world)
        eng.close()
    with open(os.path.join(outdir, "overlap_{}.json".format(rank)), "w") as f:
        json.dump(out, f)
    shutdown(ctx)


def test_async_hops_overlap_validation(tmp_path):
    world = 2
    mp.spawn(_overlap_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
             join=True)
    per = [json.load(open(tmp_path / "overlap_{}.json".format(r))) for r in range(world)]
    for r, o in enumerate(per):
        a, l = o["async"], o["lockstep"]
        print(r, o)
        assert a["bytes"] > 0 and a["nhops"] > 0
        # the forced 0.1 s transfers hide behind the receiver's validation
        assert a["exposed"] < 0.01 * a["wall"], a
        assert a["overlap"] > 0.5 * 0.1 * a["nhops"] / 2, a
        # the lock-step runtime pays for them
        assert l["exposed"] > 0.1, l
    assert per[0]["async"]["wall"] < per[0]["lockstep"]["wall"]


# ---------------------------------------------------------------------------
def test_resident_jobs_skip_state_copies(monkeypatch):
    """World 1, 4 partitions: after the first sub-epoch every config stays
    resident in its working row; only part_of_row changes (the lock-step
    runtime copies every state in and out every round)."""
    monkeypatch.setenv("CEREBRO_BACKEND", "torch")
    monkeypatch.setenv("CEREBRO_QUIET", "1")
    from cerebro_ds_kpgi_amd.parallel import DistContext
    counts = {}
    states = {}
    for runtime in ("async", "lockstep"):
        eng = _engine(DistContext(), 4, 4, scheduler="rotation", runtime=runtime)
        eng.run(2)
        grp = next(iter(eng.groups.values()))
        counts[runtime] = grp.n_loads
        states[runtime] = {m: eng.group_of[m].state_row(m).clone() for m in range(4)}
        _pairs_once(eng, 4, 4)
        eng.close()
    assert counts["async"] == 4                    # the first round only
    assert counts["lockstep"] == 4 * 8
    for m in range(4):                             # same visits; row order = float noise
        torch.testing.assert_close(states["async"][m], states["lockstep"][m],
                                   rtol=2e-2, atol=2e-3)


def _greedy_fault_worker(rank, world, port, outdir):
    _env(rank, world, port)
    from cerebro_ds_kpgi_amd.parallel import init_distributed, shutdown
    ctx = init_distributed(device_type="cpu")
    eng = _engine(ctx, 4, 2, scheduler="greedy", runtime="async", fault_inject="1:0:soft")
    eng.run(2)
    _pairs_once(eng, 4, 2 * world)
    fin = all(bool(torch.isfinite(eng.group_of[m].state_row(m)).all())
              for m in range(4) if eng.holder[m] == rank)
    if rank == 0:
        with open(os.path.join(outdir, "out.json"), "w") as f:
            json.dump({"failures": eng.failures, "finite": fin,
                       "epochs": {str(k): len(v["valid_loss"])
                                  for k, v in eng.mst_state.items()}}, f)
    eng.close()
    shutdown(ctx)


def test_async_greedy_requeues_soft_fault(tmp_path):
    world = 2
    mp.spawn(_greedy_fault_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
             join=True)
    with open(tmp_path / "out.json") as f:
        out = json.load(f)
    assert out["failures"] and all(f["rank"] == 1 for f in out["failures"])
    assert out["finite"] and set(out["epochs"].values()) == {2}


# ---------------------------------------------------------------------------
def _ring_worker(rank, world, port, outdir, job_s, hop_s):
    _env(rank, world, port)
    from cerebro_ds_kpgi_amd.parallel import init_distributed, shutdown
    ctx = init_distributed(device_type="cpu")
    eng = _engine(ctx, world, 1, scheduler="rotation", runtime="async", trace=True,
                  hop_check=True, sim_job_seconds=job_s, sim_hop_seconds=hop_s,
                  logs_root=outdir)
    ctx.barrier()
    eng.run(1)
    _pairs_once(eng, world, world)
    with open(os.path.join(outdir, "ring_{}.json".format(rank)), "w") as f:
        json.dump({"spans": eng.hop_spans, "bytes": eng.hop_bytes,
                   "groups": eng.hop_groups}, f)
    eng.close()
    shutdown(ctx)


def _metrics(outdir, kind):
    return [r for r in (json.loads(l) for l in open(os.path.join(outdir, "metrics.jsonl")))
            if r.get("kind") == kind]


def test_async_rotation_ring_shift_is_one_phase(tmp_path, monkeypatch):
    """8 ranks, rotation: at every sub-epoch boundary each rank sends its
    model to the next rank and receives one from the previous.  On the ONE
    hop communicator the shift runs as one phase only if every rank posts
    the boundary's send and receive in ONE ``batch_isend_irecv`` group (the
    coordinator publishes the shift as one burst); posted as two groups, a
    rank's receive from its predecessor sits in front of its own send and
    the shift chains through the ring.  Checked from the hop records (not
    from wall-clock overlap): on every rank, every group
    holds exactly one send and one receive, and there is one group per
    boundary.  The forced link time (0.25 s) is long against scheduler
    jitter, so the coordinator's hold margin (2 x the transfer time) keeps a
    boundary's hops in one burst on a loaded host.  The mean number of a
    boundary's transfers in flight (8 = one phase, 1 = a chain) is printed
    as a diagnostic only.

    Runs under RCCL's matching rules (tag-blind, the default: gloo pairs the
    operations per peer in posting order, as RCCL does)."""
    world = 8
    monkeypatch.delenv("CER_HOP_TAGS", raising=False)
    mp.spawn(_ring_worker, args=(world, _free_port(), str(tmp_path), [0.05], 0.25),
             nprocs=world, join=True)
    sends = []
    for r in range(world):
        d = json.load(open(tmp_path / "ring_{}.json".format(r)))
        assert d["bytes"] > 0
        groups = collections.defaultdict(list)
        for sp in d["spans"]:
            groups[(sp[0], sp[1])].append(sp[2])
        nb = sum(1 for sp in d["spans"] if sp[2] == "send")
        assert nb == world - 1, (r, nb)                      # 8 rounds = 7 boundaries
        assert d["groups"] == len(groups) == nb, (r, d["groups"], len(groups), nb)
        for key, dirs in groups.items():
            assert sorted(dirs) == ["recv", "send"], (r, key, dirs)
        sends.append(sorted((sp[0], sp[1]) for sp in d["spans"] if sp[2] == "send"))
    conc = []
    for k in range(world - 1):
        spans = [sd[k] for sd in sends]
        t0 = min(a for a, _ in spans)
        t1 = max(b for _, b in spans)
        conc.append(sum(b - a for a, b in spans) / (t1 - t0))
    print("ring-shift concurrency per boundary (diagnostic):", [round(c, 2) for c in conc])
    # the per-hop telemetry: one record per hop endpoint
    recs = _metrics(tmp_path, "hop")
    assert len(recs) == 2 * world * (world - 1)
    for rec in recs:
        assert set(rec) >= {"seq", "rank", "dir", "model", "peer", "bytes", "t_post",
                            "post_to_arrival_us", "hold_us"}, rec
        assert rec["bytes"] > 0 and rec["post_to_arrival_us"] >= 0.25e6 * 0.9
    assert len(_metrics(tmp_path, "hop_hold")) == 1


def test_rotation_hold_is_not_bounded_by_a_straggler(tmp_path, monkeypatch):
    """one forced straggler (config 3 trains 4x longer
    than the others, so whichever rank holds it is slow in that round) does
    not hold the other ranks' hops back.  The coordinator holds a hop only
    while a rank within its hold margin (2 x the measured transfer time) of
    the median job time is still training; round 5's rule held every hop
    while ANY computing rank was unfinished, up to 0.2 x the mean job time
    (here ~80 ms against a ~10-30 ms margin).  Every hop's hold (from the
    metrics records) stays within the margin plus scheduling slack."""
    world = 8
    monkeypatch.delenv("CER_HOP_TAGS", raising=False)
    jobs = [0.3] * world
    jobs[3] = 1.2
    mp.spawn(_ring_worker, args=(world, _free_port(), str(tmp_path), jobs, 0.005),
             nprocs=world, join=True)
    hold = _metrics(tmp_path, "hop_hold")[0]
    recv = [r for r in _metrics(tmp_path, "hop") if r["dir"] == "recv"]
    assert len(recv) == world * (world - 1)
    worst = max(r["hold_us"] for r in recv) / 1e6
    margin = hold["margin_us_max"] / 1e6
    print("hold max {:.4f}s mean {:.4f}s margin {:.4f}s".format(
        worst, hold["hold_us_mean"] / 1e6, margin))
    assert margin < 0.05, hold
    assert worst <= margin + 0.04, (worst, margin)


# ---------------------------------------------------------------------------
def _greedy8_worker(rank, world, port, outdir):
    _env(rank, world, port)
    from cerebro_ds_kpgi_amd.parallel import init_distributed, shutdown
    ctx = init_distributed(device_type="cpu")
    # 8 configs on 8 ranks x 1 partition, greedy: every boundary is an
    # arbitrary permutation (not a ring), every hop digest-verified
    eng = _engine(ctx, world, 1, scheduler="greedy", runtime="async", hop_check=True,
                  sim_job_seconds=[0.01, 0.03, 0.02, 0.05, 0.01, 0.04, 0.02, 0.03])
    ctx.barrier()
    eng.run(2)
    _pairs_once(eng, world, world)
    fin = all(bool(torch.isfinite(eng.group_of[m].state_row(m)).all())
              for m in range(world) if eng.holder[m] == rank)
    with open(os.path.join(outdir, "g_{}.json".format(rank)), "w") as f:
        json.dump({"bytes": eng.hop_bytes, "groups": eng.hop_groups, "finite": fin,
                   "epochs": {str(k): len(v["valid_loss"]) for k, v in eng.mst_state.items()}},
                  f)
    eng.close()
    shutdown(ctx)


def test_async_greedy_permutations_hop_checked(tmp_path):
    """8 ranks, greedy MOP with heterogeneous job lengths: hops form
    arbitrary permutations published at arbitrary times; with the debug
    digest check (``CER_HOP_CHECK=1`` semantics) every transfer arrives
    intact on the single hop communicator, and both epochs complete."""
    world = 8
    mp.spawn(_greedy8_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
             join=True)
    per = [json.load(open(tmp_path / "g_{}.json".format(r))) for r in range(world)]
    assert sum(d["bytes"] for d in per) > 0
    assert all(d["finite"] for d in per)
    assert set(per[0]["epochs"].values()) == {2}
