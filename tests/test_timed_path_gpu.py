"""The bench's timed path against the fp32 oracle.

``bench.py`` times ``MOPEngine.run_steps`` on 8 ResNet-50 configs at batch
32 packed into ONE G = 8 pack on one GPU, with every production switch on:
HIP-graph replay of the step, the side-stream batch of weight gradients
(fires at G x B >= 64), lazy residual gradients, BN links, the stem prep
launch, the uniform-K GEMM kernels and the optimizer-written HL weight image
(``runtime/arena.py`` ``Arena.whl``).  This test trains exactly that engine
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
    from cerebro_ds_kpgi_amd.parallel import DistContext
    from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine
    from cerebro_ds_kpgi_amd.selection import get_msts
    set_backend(backend_name)
    msts = get_msts(dict(cat.param_grid_scalability))          # 8 configs, bs 32
    assert len(msts) == 8 and {m["batch_size"] for m in msts} == {32}
    n_train = per_round * 32
    eng = MOPEngine(msts, DistContext(), EngineOptions(
        slots_per_gpu=8, scheduler="rotation", n_train=n_train, n_valid=32,
        compute_dtype="fp32", use_graphs=True, verbose=False, ckpt_every="none", seed=2018))
    counts0 = dict(_hip.HL_COUNTS)
    eng.run_steps(steps, per_round)
    torch.cuda.synchronize()
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
    hip, info = _train("hip")
    ref, _ = _train("torch")
    print("timed path:", info)
    # the production switches really ran: one G = 8 pack, a replayed step
    # graph, HL operands, the HL weight image
    assert info["G"] == 8 and info["graph"] and info["whl"], info
    assert info["hl"]["x"] > 0 and info["hl"]["dy"] > 0, info
    assert sorted(hip) == sorted(ref) and len(hip) == 8
    worst = 0.0
    for key in hip:
        h = torch.tensor(hip[key], dtype=torch.float64)
        r = torch.tensor(ref[key], dtype=torch.float64)
        assert len(h) == len(r) == 5, (key, len(h), len(r))
        assert torch.isfinite(h).all()
        dev = ((h - r).abs() / r[0]).max().item()
        worst = max(worst, dev)
        print(key, "hip", [round(v, 4) for v in h.tolist()], "ref",
              [round(v, 4) for v in r.tolist()], "dev %.2e" % dev)
    assert worst < 2e-2, worst
