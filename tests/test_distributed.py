"""Multi-process MOP on CPU (gloo, world_size 2) — BASELINE config 1.

The same 4-config tiny-CNN MOP run is executed (a) in one process holding all
4 partitions and (b) in two processes holding 2 partitions each, where every
sub-epoch boundary ships models across ranks by point-to-point send/recv.
Model hopping must be transparent: final weights, optimizer state and the
per-epoch metrics must agree.
"""

import collections
import json
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _msts():
    from cerebro_ds_kpgi_amd.config import catalog as cat
    from cerebro_ds_kpgi_amd.selection import get_msts
    base = get_msts(cat.param_grid_tiny)
    out = []
    for i, lr in enumerate([1e-3, 3e-3, 1e-2, 2e-3]):
        m = dict(base[0])
        m["learning_rate"] = lr
        out.append(m)
    return out


def _run(rank, world, port, outdir, slots, scheduler, hop_opt, runtime="auto"):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                       "CEREBRO_BACKEND": "torch", "CEREBRO_QUIET": "1"})
    torch.set_num_threads(1)
    from cerebro_ds_kpgi_amd.parallel import init_distributed, shutdown
    from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine
    ctx = init_distributed(device_type="cpu")
    eng = MOPEngine(_msts(), ctx, EngineOptions(
        n_train=64, n_valid=16, compute_dtype="fp32", slots_per_gpu=slots, scheduler=scheduler,
        hop_optimizer_state=hop_opt, verbose=False, ckpt_every="none", runtime=runtime,
        models_root=os.path.join(outdir, "models"), logs_root=os.path.join(outdir, "logs")))
    eng.run(2)
    states = {}
    for m in range(len(eng.msts)):
        if eng.holder[m] == rank:
            grp = eng.group_of[m]
            states[m] = grp.state_row(m).clone()
    torch.save(states, os.path.join(outdir, "states_{}.pt".format(rank)))
    if rank == 0:
        with open(os.path.join(outdir, "mst_state.json"), "w") as f:
            json.dump({str(k): v for k, v in eng.mst_state.items()}, f)
        with open(os.path.join(outdir, "hops.json"), "w") as f:
            json.dump({"hop_bytes": eng.hop_bytes}, f)
    eng.close()
    shutdown(ctx)


def _launch(tmp, world, slots, scheduler="rotation", hop_opt=True, runtime="auto"):
    port = _free_port()
    if world == 1:
        _run(0, 1, port, tmp, slots, scheduler, hop_opt, runtime)
    else:
        mp.spawn(_run, args=(world, port, tmp, slots, scheduler, hop_opt, runtime), nprocs=world,
                 join=True)
    states = {}
    for r in range(world):
        states.update(torch.load(os.path.join(tmp, "states_{}.pt".format(r)), weights_only=True))
    with open(os.path.join(tmp, "mst_state.json")) as f:
        mst_state = json.load(f)
    with open(os.path.join(tmp, "hops.json")) as f:
        hops = json.load(f)
    return states, mst_state, hops


# rotation runs on the asynchronous runtime (data-flow rounds, hops on their
# own thread) and must reproduce the single-process visit order; the greedy
# case pins the lock-step runtime, whose greedy plan is deterministic (the
# asynchronous greedy order depends on event timing: test_async_runtime)
@pytest.mark.parametrize("scheduler,hop_opt,runtime", [("rotation", True, "async"),
                                                       ("greedy", False, "lockstep")])
def test_two_rank_mop_matches_single_process(tmp_path, scheduler, hop_opt, runtime):
    a = tmp_path / "one"
    b = tmp_path / "two"
    a.mkdir()
    b.mkdir()
    s1, m1, _ = _launch(str(a), 1, 4, scheduler, hop_opt, runtime)
    s2, m2, hops = _launch(str(b), 2, 2, scheduler, hop_opt, runtime)
    assert hops["hop_bytes"] > 0                       # models really crossed ranks
    assert sorted(s1) == sorted(s2) == [0, 1, 2, 3]
    # packing 4 vs 2 configs per process changes CPU grouped-conv blocking, so
    # agreement is to float noise (amplified by Adam's 1/sqrt(v)); a mis-routed
    # model would differ by O(1).  Bitwise hop exactness: test_hop_bitwise.
    # With per-sub-epoch Adam resets (hop_opt=False) every reset step moves each
    # weight by ~lr*sign(g), so float noise in near-zero gradients is amplified
    # to O(lr) weight differences; tolerances reflect that.
    for m in s1:
        torch.testing.assert_close(s1[m], s2[m], rtol=2e-2, atol=2e-3 if hop_opt else 1e-1)
    for k in m1:
        assert m1[k]["train_loss"] == pytest.approx(m2[k]["train_loss"], rel=1e-3 if hop_opt else 3e-2)
        assert len(m1[k]["valid_loss"]) == 2


def _hop_worker(rank, world, port, outdir):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    from cerebro_ds_kpgi_amd.parallel import init_distributed, shutdown
    from cerebro_ds_kpgi_amd.parallel.hop import (execute_moves, plan_moves, validate_plan,
                                                  warm_p2p)
    ctx = init_distributed(device_type="cpu")
    assert warm_p2p(world, rank, "cpu") == world - 1
    # 6 models on 3 ranks, arbitrary permutation incl. 2-cycles and a 3-cycle
    holder = {m: m % world for m in range(6)}
    dest = {0: 1, 1: 0, 2: 0, 3: 2, 4: 1, 5: 2}
    moves = plan_moves(holder, dest)
    validate_plan(moves, world)
    g = torch.Generator().manual_seed(7)
    rows = {m: torch.randn(1000, generator=g) for m in range(6)}
    recv = {m: torch.full((1000,), float("nan")) for m in range(6)}
    execute_moves(moves, rank, lambda m: rows[m], lambda m: recv[m], check=True)
    got = {m: recv[m] for m in range(6) if dest[m] == rank and holder[m] != rank}
    ok = all(torch.equal(got[m], rows[m]) for m in got)
    # debug hop check: a send buffer that changes while "in flight" (here: a
    # different tensor the second time it is asked for) must be caught
    from cerebro_ds_kpgi_amd.parallel.hop import HopChecksumError
    asked = collections.Counter()

    def racy(m):
        asked[m] += 1
        return rows[m] if asked[m] == 1 or rank != 0 else rows[m] + 1.0
    caught = 0
    try:
        execute_moves(moves, rank, racy, lambda m: recv[m], check=True)
    except HopChecksumError:
        caught = 1
    with open(os.path.join(outdir, "hop_{}.txt".format(rank)), "w") as f:
        f.write("{} {} {}".format(int(ok), len(got), caught))
    shutdown(ctx)


def test_hop_bitwise(tmp_path):
    world = 3
    mp.spawn(_hop_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    total = caught = 0
    for r in range(world):
        ok, n, c = open(tmp_path / "hop_{}.txt".format(r)).read().split()
        assert ok == "1"
        total += int(n)
        caught += int(c)
    assert total == 4   # models 0, 1, 2, 4 change rank; 3 and 5 stay
    assert caught >= 1  # rank 0's racing sends are detected by their receivers


def test_checkpoint_layout_and_resume(tmp_path):
    """CTQ checkpoint layout ({i}_{mst_str} + .opt + .json), loadable as a
    flat float32 weight blob and restorable into an arena."""
    from cerebro_ds_kpgi_amd.runtime.checkpoint import host_to_state, read_checkpoint
    from cerebro_ds_kpgi_amd.utils.keys import model_key
    os.environ["CEREBRO_BACKEND"] = "torch"
    from cerebro_ds_kpgi_amd.parallel import init_distributed
    from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine
    ctx = init_distributed(device_type="cpu")
    msts = _msts()
    eng = MOPEngine(msts, ctx, EngineOptions(
        n_train=64, n_valid=16, compute_dtype="fp32", slots_per_gpu=4, verbose=False,
        models_root=str(tmp_path / "models"), logs_root=str(tmp_path / "logs")))
    eng.run(1)
    eng.close()
    for i, mst in enumerate(msts):
        path = tmp_path / "models" / model_key(i, mst)
        assert path.exists() and (tmp_path / "models" / (model_key(i, mst) + ".opt")).exists()
        w, opt, meta = read_checkpoint(str(path))
        grp = eng.group_of[i]
        assert w.dtype.name == "float32" and w.size == sum(s.numel for s in grp.layout.specs)
        assert meta["epoch"] == 1 and meta["mst"]["learning_rate"] == mst["learning_rate"]
        row = torch.zeros_like(grp.state_row(i))
        host_to_state(grp.layout, w, opt, row)
        torch.testing.assert_close(row, grp.state_row(i))
    assert (tmp_path / "logs" / "jobs_info.pkl").exists()
    assert (tmp_path / "logs" / "models_info.pkl").exists()
