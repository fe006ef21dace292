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
def _ring_worker(rank, world, port, outdir):
    _env(rank, world, port)
    from cerebro_ds_kpgi_amd.parallel import init_distributed, shutdown
    ctx = init_distributed(device_type="cpu")
    eng = _engine(ctx, world, 1, scheduler="rotation", runtime="async", trace=True,
                  hop_check=True, sim_job_seconds=[0.05], sim_hop_seconds=0.1)
    ctx.barrier()
    eng.run(1)
    _pairs_once(eng, world, world)
    with open(os.path.join(outdir, "ring_{}.json".format(rank)), "w") as f:
        json.dump({"spans": eng.hop_spans, "bytes": eng.hop_bytes,
                   "groups": eng.hop_groups}, f)
    eng.close()
    shutdown(ctx)


def test_async_rotation_ring_shift_is_one_phase(tmp_path, monkeypatch):
    """8 ranks, rotation: at every sub-epoch boundary each rank sends its
    model to the next rank and receives one from the previous.  With a
    forced 0.1 s per transfer a boundary's eight sends overlap (one phase,
    ~0.1 s), instead of chaining through the ring (~0.8 s).  On the ONE hop
    communicator this needs the boundary's send and receive in one group on
    every rank: the coordinator publishes the ring shift as one burst and
    each rank posts it as one ``batch_isend_irecv`` group.  Measured as the
    mean number of a boundary's transfers in flight (8 = one phase, 1 = a
    chain) and as groups per rank (one per boundary).

    Runs under RCCL's matching rules (tag-blind, the default: gloo pairs the
    operations per peer in posting order, as RCCL does)."""
    world = 8
    monkeypatch.delenv("CER_HOP_TAGS", raising=False)
    # a timing property on a shared CPU host: one retry when a scheduling
    # hiccup splits the shifts (the chained service stays ~1-2.5 every time)
    err = None
    for attempt in range(3):
        try:
            conc = _ring_run(tmp_path / str(attempt), world)
        except AssertionError as e:          # a straggler split a boundary's group
            err, conc = e, [0.0]
            continue
        err = None
        print("ring-shift concurrency per boundary:", [round(c, 2) for c in conc])
        if statistics.median(conc) >= 3.0:
            break
    if (err is not None or statistics.median(conc) < 3.0) and \
            os.getloadavg()[0] > 0.5 * (os.cpu_count() or 1):
        # 8 ranks time-sliced with other test workers cannot show the overlap
        pytest.skip("host loaded (loadavg {:.1f}): {}".format(os.getloadavg()[0], err or conc))
    if err is not None:
        raise err
    # (~7.6-7.9 on an idle host: every boundary is one phase)
    assert statistics.median(conc) >= 3.0, conc


def _ring_run(tmp_path, world):
    tmp_path.mkdir(parents=True, exist_ok=True)
    mp.spawn(_ring_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    sends = []
    for r in range(world):
        d = json.load(open(tmp_path / "ring_{}.json".format(r)))
        assert d["bytes"] > 0
        # mostly one group per boundary (send and receive together; a late
        # straggler past the coordinator's hold splits one now and then);
        # posted one by one they would be 2 per boundary
        nsend = sum(1 for s in d["spans"] if s[2] == "send")
        assert d["groups"] < 2 * nsend, (r, d["groups"], nsend)
        sends.append(sorted((s[0], s[1]) for s in d["spans"] if s[2] == "send"))
    nb = min(len(s) for s in sends)
    assert nb >= world - 1, [len(s) for s in sends]
    conc = []
    for k in range(nb):
        spans = [s[k] for s in sends]
        t0 = min(a for a, _ in spans)
        t1 = max(b for _, b in spans)
        # mean number of this boundary's transfers in flight: ~1 when they
        # chain through the ring, up to 8 when they run as one phase (start
        # skew between ranks -- the rotation is a data flow, not a barrier --
        # only lowers it)
        conc.append(sum(b - a for a, b in spans) / (t1 - t0))
    return conc


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
