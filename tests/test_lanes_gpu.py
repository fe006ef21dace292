"""Concurrent pack groups (runtime/async_mop._Lanes): a batch whose pack
groups are all past their warm-up replays each group's step graph on its
lane's stream, at the same time.  The result must equal the serial run (all
groups forced onto one lane) up to the fp32 atomic order of the weight
gradients."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(one_lane):
    from cerebro_ds_kpgi_amd.parallel import init_distributed
    from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine
    msts = [{"learning_rate": lr, "lambda_value": 1e-4, "batch_size": bs, "model": "resnet18"}
            for bs in (8, 16) for lr in (1e-3, 1e-4)]
    eng = MOPEngine(msts, init_distributed(), EngineOptions(
        n_train=64, n_valid=16, slots_per_gpu=4, verbose=False, ckpt_every="none",
        shuffle=False, scheduler="rotation", runtime="async"))
    if one_lane:
        for g in eng.groups.values():
            g.lane = 0
    assert len({g.lane for g in eng.groups.values()}) == (1 if one_lane else 2)
    eng.run(2)
    torch.cuda.synchronize()
    out = {k: g.home.state.clone() for k, g in eng.groups.items()}
    lanes = eng.lane_batches
    eng.close()
    return out, lanes


def test_lanes_match_serial_groups():
    conc, n_conc = _run(False)
    ser, _ = _run(True)
    assert n_conc > 0, "no batch ran its groups on lane streams"
    for k in ser:
        assert torch.isfinite(conc[k]).all()
        torch.testing.assert_close(conc[k], ser[k], rtol=2e-4, atol=2e-5)
