"""Stream / hardware-queue budget (profiles/r5_stream_budget.md).

The headline engine's active streams per workload shape are counted by
``MOPEngine.stream_budget``; lanes default to 4 (one GPU) and, at world > 1, never
push the hop's streams out of the 4 hardware queues.  CPU: the engine is
built on gloo ranks (the accounting does not depend on the device)."""

import json
import os

import torch.multiprocessing as mp

from test_distributed import _free_port


def _budget_worker(rank, world, port, outdir):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                       "CEREBRO_BACKEND": "torch", "CEREBRO_QUIET": "1"})
    from cerebro_ds_kpgi_amd.config import catalog as cat
    from cerebro_ds_kpgi_amd.parallel import init_distributed, shutdown
    from cerebro_ds_kpgi_amd.runtime.engine import LANES, EngineOptions, MOPEngine
    from cerebro_ds_kpgi_amd.selection import get_msts
    ctx = init_distributed(device_type="cpu")
    msts = get_msts(cat.param_grid_scalability)             # the 8 headline configs
    out = {"LANES": LANES}
    eng = MOPEngine(msts, ctx, EngineOptions(n_train=32, n_valid=32, verbose=False,
                                             ckpt_every="none"))
    out["headline"] = sorted(eng.stream_budget())
    out["lanes_default"] = eng.effective_lanes(4)
    eng.close()
    eng = MOPEngine(msts, ctx, EngineOptions(n_train=32, n_valid=32, verbose=False,
                                             ckpt_every="none", lanes=4))
    out["lanes4_4groups"] = eng.effective_lanes(4)
    out["g1"] = sorted(eng.stream_budget({k: 1 for k in eng.groups}))
    eng.close()
    if rank == 0:
        with open(os.path.join(outdir, "budget.json"), "w") as f:
            json.dump(out, f)
    shutdown(ctx)


def test_headline_stream_budget_world2(tmp_path):
    world = 2
    mp.spawn(_budget_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    out = json.load(open(tmp_path / "budget.json"))
    # the default asks for 4 lanes (world 1); at world > 1 they are clamped
    assert out["LANES"] == 4 and out["lanes_default"] == 1
    # 4 configs per GPU (N = 2): compute, branch, side wgrad, hop, RCCL
    assert out["headline"] == ["branch", "compute", "hop", "rccl_hop", "side_wgrad"]
    # one config per GPU (the N = 8 shape): no side batch -> 4 = the queues
    assert out["g1"] == ["branch", "compute", "hop", "rccl_hop"]
    # asked-for lanes are clamped at world > 1 (hop + RCCL keep their queues)
    assert out["lanes4_4groups"] == 1


def test_world1_budget_and_lanes():
    os.environ["CEREBRO_BACKEND"] = "torch"
    from cerebro_ds_kpgi_amd.config import catalog as cat
    from cerebro_ds_kpgi_amd.parallel import DistContext
    from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine
    from cerebro_ds_kpgi_amd.selection import get_msts
    eng = MOPEngine(get_msts(cat.param_grid_scalability)[:2], DistContext(),
                    EngineOptions(n_train=32, n_valid=32, verbose=False, ckpt_every="none",
                                  lanes=3, slots_per_gpu=2))
    assert eng.effective_lanes(4) == 3 and eng.effective_lanes(2) == 2
    b = eng.stream_budget()
    assert "hop" not in b and "compute" in b and "side_wgrad" in b
    eng.close()
