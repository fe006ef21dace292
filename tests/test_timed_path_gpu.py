"""The bench's timed path against the fp32 oracle.

``bench.py`` times ``MOPEngine.run_steps`` on 8 ResNet-50 configs at batch
32 packed into ONE G = 8 pack on one GPU, with every production switch on:
HIP-graph replay of the step, the side-stream batch of weight gradients
(fires at G x B >= 64), lazy residual gradients, BN links, the stem prep
launch and the uniform-K GEMM kernels (the optimizer-written HL weight
image, ``runtime/arena.py`` ``Arena.whl``, is on for packs of at most
``group.WHL_MAX_G`` configs: the one-config shape).  This test trains exactly that engine
for 100 steps (5 rounds of 20, the bench's ``--steps_per_round``) with the
HIP backend and with ``--backend torch`` (the PyTorch / MIOpen oracle,
``/root/reference/cerebro_gpdb/run_pytorchddp.py:285-355``: the torch train
step is the numerical oracle) from the same seeded init and
the same seeded partitions, and compares each config's per-round mean train
loss: within 2e-2 of the initial loss level, the window bound of
``test_fp32_gpu.test_resnet50_trajectory_fp32_hip_vs_oracle``.
"""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _train(backend_name, steps=100, per_round=20):
    from cerebro_ds_kpgi_amd.config import catalog as cat
    from cerebro_ds_kpgi_amd.ops import set_backend
    from cerebro_ds_kpgi_amd.ops import _hip
    from cerebro_ds_kpgi_amd.parallel import init_distributed
    from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine
    from cerebro_ds_kpgi_amd.selection import get_msts
    import time
    t0 = time.time()
    set_backend(backend_name)
    msts = get_msts(dict(cat.param_grid_scalability))          # 8 configs, bs 32
    assert len(msts) == 8 and {m["batch_size"] for m in msts} == {32}
    n_train = per_round * 32
    ctx = init_distributed()                    # one process, cuda:0 (as bench.py)
    assert ctx.device.type == "cuda"
    eng = MOPEngine(msts, ctx, EngineOptions(
        slots_per_gpu=8, scheduler="rotation", n_train=n_train, n_valid=32,
        compute_dtype="fp32", use_graphs=True, verbose=False, ckpt_every="none", seed=2018))
    counts0 = dict(_hip.HL_COUNTS)
    print("[{}] engine ready {:.1f}s".format(backend_name, time.time() - t0), flush=True)
    for r in range(steps // per_round):
        eng.run_steps(per_round, per_round, epoch_start=1 + r)
        torch.cuda.synchronize()
        print("[{}] round {} done {:.1f}s".format(backend_name, r, time.time() - t0), flush=True)
    curves = {}
    for key, jobs in eng.models_info.items():
        js = sorted(jobs, key=lambda j: (j["epoch"], j["subepoch"]))
        curves[key] = [j["loss_train"] for j in js]
    info = {"hl": {k: _hip.HL_COUNTS[k] - counts0.get(k, 0) for k in _hip.HL_COUNTS}}
    if backend_name == "hip":
        grp = next(iter(eng.groups.values()))
        w = next(iter(grp._work.values()))
        info["G"] = w.G
        info["graph"] = w.graph is not None
        info["whl"] = w.arena.whl is not None
    eng.close()
    set_backend("hip")
    return curves, info


def test_bench_timed_path_trajectory_vs_oracle():
    import faulthandler
    import sys
    faulthandler.dump_traceback_later(150, repeat=True, file=sys.stderr)
    try:
        _check()
    finally:
        faulthandler.cancel_dump_traceback_later()


def _check():
    hip, info = _train("hip")
    ref, _ = _train("torch")
    print("timed path:", info)
    # the production switches really ran: one G = 8 pack, a replayed step
    # graph, HL operands, the HL weight image
    from cerebro_ds_kpgi_amd.runtime.group import WHL_MAX_G
    assert info["G"] == 8 and info["graph"] and info["whl"] == (8 <= WHL_MAX_G), info
    assert info["hl"]["x"] > 0 and info["hl"]["dy"] > 0, info
    assert sorted(hip) == sorted(ref) and len(hip) == 8
    # lr <= 1e-4: the window bound of the eager trajectory test (2e-2; these
    # configs measure 2e-5 - 7e-3 on the GPU box).  lr = 1e-3 starts at a loss
    # of ~10.9 on a 1000-class head and is chaotic: two fp32 implementations
    # of the same step drift apart by rounding alone (1.5e-2 - 1.9e-2
    # measured), so its bound is 5e-2
    worst = {}
    for key in hip:
        h = torch.tensor(hip[key], dtype=torch.float64)
        r = torch.tensor(ref[key], dtype=torch.float64)
        assert len(h) == len(r) == 5, (key, len(h), len(r))
        assert torch.isfinite(h).all()
        dev = ((h - r).abs() / r[0]).max().item()
        lr = float(key.split("learning_rate:")[1].split(",")[0])
        bound = 2e-2 if lr <= 1e-4 else 5e-2
        worst[key] = (dev, bound)
        print(key, "hip", [round(v, 4) for v in h.tolist()], "ref",
              [round(v, 4) for v in r.tolist()], "dev %.2e (bound %.0e)" % (dev, bound))
    assert all(d < b for d, b in worst.values()), worst
