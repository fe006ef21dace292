"""Multi-rank MA and DDP baselines on gloo.

* MA: after every epoch all ranks hold the image-count-weighted mean of the
  per-rank weights (reference merge ``madlib_keras_wrapper.py:63-116``),
  including with unequal counts;
* MA and DDP coalesce their collectives: one all-reduce per merge and one
  per gradient bucket, over all G packed config rows;
* DDP: the gradient after the bucketed, backward-overlapped all-reduce equals
  the single-process gradient of the concatenated batch (BN-free model: the
  reference's DDP keeps BatchNorm statistics per rank), with one bucket per
  mark (several all-reduces in flight during backward);
* a 2-rank DDPEngine run keeps every rank's weights identical.
"""

import os

import pytest
import torch
import torch.multiprocessing as mp

from test_distributed import _free_port


def _env(rank, world, port):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                       "CEREBRO_BACKEND": "torch", "CEREBRO_QUIET": "1"})
    torch.set_num_threads(1)


def _count_all_reduce():
    """Count torch.distributed.all_reduce calls from here on (this process)."""
    import torch.distributed as dist
    calls = [0]
    orig = dist.all_reduce

    def counted(*a, **k):
        calls[0] += 1
        return orig(*a, **k)
    dist.all_reduce = counted
    return calls


def _tiny_msts(n):
    return [{"model": "tinycnn", "batch_size": 8, "learning_rate": 1e-3 * (i + 1),
             "lambda_value": 1e-4} for i in range(n)]


def _ma_worker(rank, world, port, outdir):
    _env(rank, world, port)
    from cerebro_ds_kpgi_amd.parallel import init_distributed, shutdown
    from cerebro_ds_kpgi_amd.runtime.baselines import MAEngine
    from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions
    ctx = init_distributed(device_type="cpu")
    eng = MAEngine(_tiny_msts(2), ctx, EngineOptions(n_train=32, n_valid=16,
                                                     compute_dtype="fp32", verbose=False))
    eng.keep_pre_average = True
    eng.run(1)
    grp = next(iter(eng.groups.values()))
    w = grp._work[2]
    out = {"pre": eng.pre_average, "post": w.arena.master.detach().clone()}
    # unequal image counts: rank r contributes count r + 1
    g = torch.Generator().manual_seed(100 + rank)
    w.arena.master.copy_(torch.randn(w.arena.master.shape, generator=g))
    out["x"] = w.arena.master.detach().clone()
    calls = _count_all_reduce()
    eng._average(w, rank + 1)
    out["collectives"] = torch.tensor(calls[0])
    out["avg"] = w.arena.master.detach().clone()
    torch.save(out, os.path.join(outdir, "ma_{}.pt".format(rank)))
    shutdown(ctx)


def test_ma_weighted_average_three_ranks(tmp_path):
    world = 3
    mp.spawn(_ma_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [torch.load(str(tmp_path / "ma_{}.pt".format(r)), weights_only=True)
           for r in range(world)]
    mean = sum(r["pre"] for r in res) / world                   # equal counts
    for r in res:
        torch.testing.assert_close(r["post"], mean, rtol=1e-6, atol=1e-6)
    assert not torch.equal(res[0]["pre"], res[1]["pre"])          # ranks did diverge
    want = sum((i + 1) * res[i]["x"] for i in range(world)) / sum(range(1, world + 1))
    for r in res:
        torch.testing.assert_close(r["avg"], want, rtol=1e-5, atol=1e-6)
        assert int(r["collectives"]) == 1          # one all-reduce per merge (G rows + count)


def _ddp_grad_worker(rank, world, port, outdir):
    _env(rank, world, port)
    from cerebro_ds_kpgi_amd.parallel import init_distributed, shutdown
    from cerebro_ds_kpgi_amd.models import create_model_from_mst
    from cerebro_ds_kpgi_amd.ops.loss import softmax_ce
    from cerebro_ds_kpgi_amd.runtime import Arena
    from cerebro_ds_kpgi_amd.runtime.baselines import GradBuckets
    ctx = init_distributed(device_type="cpu")
    G, B = 2, 6
    net = create_model_from_mst({"model": "sanity"})
    arena = Arena(net.layout, G, "cpu", torch.float32)
    for g in range(G):
        arena.init_model(g, 7 + g)
    net.bind(arena)
    gen = torch.Generator().manual_seed(0)
    xs = [torch.randn(B, G * 4, generator=gen) for _ in range(world)]
    ys = [torch.randint(0, 3, (G, B), generator=gen, dtype=torch.int32) for _ in range(world)]
    acc = torch.zeros(G, 4)
    # single-process reference: the concatenated batch
    loss = softmax_ce(net.forward(torch.cat(xs), True), torch.cat(ys, 1), acc, G)
    loss.sum().backward()
    want = arena.grad.clone()
    arena.grad.zero_()
    # DDP: this rank's slice, bucketed all-reduce during backward
    gb = GradBuckets(arena, world, bucket_bytes=4)
    net.grad_buckets = gb
    calls = _count_all_reduce()
    loss = softmax_ce(net.forward(xs[rank], True), ys[rank], acc, G)
    loss.sum().backward()
    in_backward = gb.n_buckets
    gb.finish()
    torch.save({"want": want, "got": arena.grad.clone(), "buckets": in_backward,
                "log": gb.bucket_log, "collectives": torch.tensor(calls[0])},
               os.path.join(outdir, "ddp_{}.pt".format(rank)))
    shutdown(ctx)


def test_ddp_bucketed_gradient_equals_large_batch(tmp_path):
    world = 2
    mp.spawn(_ddp_grad_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
             join=True)
    for r in range(world):
        res = torch.load(str(tmp_path / "ddp_{}.pt".format(r)), weights_only=True)
        torch.testing.assert_close(res["got"], res["want"], rtol=1e-5, atol=1e-7)
        assert res["buckets"] == 2                   # two marks fired inside backward
        lo_hi = res["log"]
        assert len(lo_hi) == 3 and lo_hi[-1][0] == 0  # + the tail bucket at finish()
        assert all(a[0] == b[1] for a, b in zip(lo_hi, lo_hi[1:]))   # contiguous, top-down
        # ONE all-reduce per bucket over both config rows (coalesced)
        assert int(res["collectives"]) == len(lo_hi)


def _ddp_engine_worker(rank, world, port, outdir):
    _env(rank, world, port)
    from cerebro_ds_kpgi_amd.parallel import init_distributed, shutdown
    from cerebro_ds_kpgi_amd.runtime.baselines import DDPEngine
    from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions
    ctx = init_distributed(device_type="cpu")
    eng = DDPEngine(_tiny_msts(2), ctx, EngineOptions(n_train=32, n_valid=16,
                                                      compute_dtype="fp32", verbose=False))
    eng.run(2)
    grp = next(iter(eng.groups.values()))
    torch.save({"state": grp.home.state.clone(), "work": grp._work[2].arena.params.clone(),
                "loss": [eng.mst_state[m]["train_loss"] for m in range(2)]},
               os.path.join(outdir, "eng_{}.pt".format(rank)))
    shutdown(ctx)


def test_ddp_engine_ranks_stay_identical(tmp_path):
    world = 2
    mp.spawn(_ddp_engine_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
             join=True)
    a, b = [torch.load(str(tmp_path / "eng_{}.pt".format(r)), weights_only=True)
            for r in range(world)]
    torch.testing.assert_close(a["work"], b["work"], rtol=0, atol=0)
    assert a["loss"] == b["loss"] and all(len(v) == 2 for v in a["loss"])
