"""Concurrent pack groups (runtime/async_mop._Lanes): a batch whose pack
groups are all past their warm-up replays each group's step graph on its
lane's stream, at the same time.  The result must equal the serial run (all
groups forced onto one lane) up to the run-to-run noise of the fp32 weight
gradient atomics.

That noise is measured, not assumed: two serial runs give the floor, and the
concurrent run may not differ from a serial one by more than a small multiple
of it.  A first serial run is discarded: it autotunes the kernel variants, so
the compared runs use the same kernels.  Small learning rates keep Adam from
amplifying the atomic-order noise over the epoch."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(one_lane):
    from cerebro_ds_kpgi_amd.parallel import init_distributed
    from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine
    msts = [{"learning_rate": lr, "lambda_value": 1e-4, "batch_size": bs, "model": "resnet18"}
            for bs in (8, 16) for lr in (1e-5, 1e-6)]
    eng = MOPEngine(msts, init_distributed(), EngineOptions(
        n_train=64, n_valid=16, slots_per_gpu=4, verbose=False, ckpt_every="none",
        shuffle=False, scheduler="rotation", runtime="async", lanes=2))
    if one_lane:
        for g in eng.groups.values():
            g.lane = 0
    assert len({g.lane for g in eng.groups.values()}) == (1 if one_lane else 2)
    eng.run(1)
    torch.cuda.synchronize()
    out = {k: g.home.state.clone() for k, g in eng.groups.items()}
    lanes = eng.lane_batches
    eng.close()
    return out, lanes


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


def test_lanes_match_serial_groups():
    _run(True)                      # autotune: the compared runs pick the same kernels
    ser_a, _ = _run(True)
    ser_b, _ = _run(True)
    conc, n_conc = _run(False)
    assert n_conc > 0, "no batch ran its groups on lane streams"
    for k in ser_a:
        assert torch.isfinite(conc[k]).all()
        noise = _rel(ser_b[k], ser_a[k])
        diff = _rel(conc[k], ser_a[k])
        print("group", k, "serial vs serial", noise, "lanes vs serial", diff)
        assert diff <= max(10 * noise, 1e-6), (k, diff, noise)
