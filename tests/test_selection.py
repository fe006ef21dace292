"""Grid / flag / key parity (reference ``in_rdbms_helper.py:156-235``,
``utils.py:58-86``) and the own-TPE search."""

import numpy as np
import pytest

from cerebro_ds_kpgi_amd.config import catalog as cat
from cerebro_ds_kpgi_amd.selection import get_exp_specific_msts, get_msts
from cerebro_ds_kpgi_amd.selection import hyperopt_helper as hh
from cerebro_ds_kpgi_amd.selection import tpe
from cerebro_ds_kpgi_amd.utils.cli import get_main_parser, main_prepare
from cerebro_ds_kpgi_amd.utils.keys import key2mst, model_key, mst2key, mst_2_str


def test_default_grid_order():
    msts = get_msts(cat.param_grid)
    assert len(msts) == 16
    # sorted by batch size, then (stable) by model name
    assert [m["model"] for m in msts[:8]] == ["resnet50"] * 8
    assert [m["batch_size"] for m in msts[:8]] == [32] * 4 + [256] * 4
    assert msts[0] == {"learning_rate": 1e-4, "lambda_value": 1e-4, "batch_size": 32,
                       "model": "resnet50"}


def test_scalability_grid():
    msts = get_msts(cat.param_grid_scalability)
    assert len(msts) == 8
    assert {m["learning_rate"] for m in msts} == {1e-3, 1e-4, 1e-5, 1e-6}
    assert all(m["model"] == "resnet50" and m["batch_size"] == 32 for m in msts)


def test_hetro_grid():
    msts = get_msts(cat.param_grid_hetro)
    assert len(msts) == 48
    assert sum(m["model"] == "mobilenetv2" for m in msts) == 38
    assert len(get_msts(cat.param_grid_hetro, hetro_dedub=True)) == 2


def test_flags_select_grids():
    p = get_main_parser()
    a = p.parse_args(["--criteo"])
    assert len(get_exp_specific_msts(a)) == 16
    a = p.parse_args(["--drill_down_scalability", "--run_single", "--single_mst_index", "3"])
    assert len(get_exp_specific_msts(a)) == 1
    a = p.parse_args(["--sanity"])
    assert len(get_exp_specific_msts(a)) == 8
    a = p.parse_args(["--drill_down_scalability", "--pytorchddp_sanity", "--size", "8"])
    assert all(m["batch_size"] == 4 for m in get_exp_specific_msts(a))
    a = p.parse_args(["--hyperopt"])
    assert len(get_exp_specific_msts(a)) == 4


def test_main_prepare_size1_and_sanity():
    args, msts = main_prepare(["--size", "1", "--sanity", "--drill_down_scalability"], verbose=False)
    assert args.train_name == args.valid_name == "imagenet_valid_data_packed_1"
    assert args.num_epochs == 1
    assert len(msts) == 8


def test_keys():
    mst = {"learning_rate": 1e-4, "lambda_value": 1e-4, "batch_size": 32, "model": "resnet50"}
    assert mst2key(mst) == "batch_size:32|lambda_value:0.0001|learning_rate:0.0001|model:resnet50"
    assert key2mst(mst2key(mst)) == mst
    assert mst_2_str(mst) == "learning_rate:0.0001,lambda_value:0.0001,batch_size:32,model:resnet50"
    assert model_key(3, mst).startswith("3_learning_rate:0.0001")


def test_tpe_beats_random_on_quadratic():
    space = {"x": tpe.uniform("x", -5, 5), "c": tpe.choice("c", [0, 1, 2])}

    def f(p):
        return (p["x"] - 1.5) ** 2 + (0 if p["c"] == 2 else 1)
    best, trials = tpe.fmin(f, space, 60, rng=np.random.RandomState(0), n_startup=10)
    assert f(best) < 0.3
    assert best["c"] == 2


def test_tpe_loguniform_bounds():
    space = hh.build_search_space()
    rng = np.random.RandomState(1)
    trials = tpe.Trials()
    for i in range(30):
        v = tpe.tpe_suggest(space, trials, rng, n_startup=5)
        mst = hh.Domain(space).to_mst(v)
        assert 1e-5 <= mst["learning_rate"] <= 0.1
        assert 16 <= mst["batch_size"] <= 256
        assert mst["model"] in ("resnet18", "resnet34")
        doc = trials.insert(v)
        trials.report(doc["tid"], abs(np.log10(mst["learning_rate"]) + 3))


def test_mst_eval_fn_hyperopt_contract():
    hp, msts, trials, domain, rand, opts = hh.init_hyperopt(cat.param_grid_hyperopt, None)
    assert len(msts) == 8
    fn = hh.mst_eval_fn_hyperopt(2, hp, trials, domain, 12, rand, 4)
    state = {i: {"train_loss": [1.0, 0.5], "valid_loss": [1.0, 0.7 + i * 0.01], "state": "RUNNING"}
             for i in range(8)}
    stop, upd, new = fn(state)
    assert sorted(stop) == list(range(8))
    assert len(new) == 4
    assert trials.trials[3]["loss"] == 0.73
    grid = hh.mst_eval_fn(2)
    assert sorted(grid(state)[0]) == list(range(8))


def test_sgd_matches_torch_optim():
    """Arena SGD (momentum, coupled L2) == torch.optim.SGD per configuration."""
    import torch
    from cerebro_ds_kpgi_amd.ops import set_backend
    from cerebro_ds_kpgi_amd.ops.optim import sgd_step
    from cerebro_ds_kpgi_amd.runtime.arena import Arena, ModelLayout, ParamSpec
    set_backend("torch")
    lay = ModelLayout([ParamSpec("w", (5, 3), "weight"), ParamSpec("b", (5,), "bias")])
    a = Arena(lay, 2, "cpu", torch.float32)
    for g in range(2):
        a.init_model(g, g)
        a.set_hparams(g, [0.1, 0.01][g], [1e-3, 0.0][g])
    ref = [torch.nn.Parameter(a.params[g].clone()) for g in range(2)]
    opts = [torch.optim.SGD([ref[g]], lr=[0.1, 0.01][g], momentum=0.9,
                            weight_decay=[1e-3, 0.0][g]) for g in range(2)]
    torch.manual_seed(0)
    for _ in range(4):
        gr = torch.randn_like(a.grad)
        a.grad.copy_(gr)
        sgd_step(a)
        for g in range(2):
            ref[g].grad = gr[g].clone()
            opts[g].step()
    for g in range(2):
        assert torch.allclose(a.params[g], ref[g].detach(), atol=1e-6)


def test_weight_blob_formats_roundtrip():
    """MADlib-wrapper byte formats + arena row <-> nd weights."""
    import numpy as np
    import torch
    from cerebro_ds_kpgi_amd.models import create_model_from_mst
    from cerebro_ds_kpgi_amd.runtime import serialize as S
    from cerebro_ds_kpgi_amd.runtime.arena import Arena
    net = create_model_from_mst({"model": "tinycnn"})
    a = Arena(net.layout, 2, "cpu", torch.float32)
    a.init_model(0, 1)
    a.init_model(1, 2)
    w = S.arena_to_nd_weights(a, 1)
    blob = S.serialize_nd_weights(w)
    assert len(blob) == 4 * sum(x.size for x in w)
    back = S.deserialize_as_nd_weights(blob, S.model_shapes(net.layout))
    assert all(np.array_equal(x, y) for x, y in zip(w, back))
    st = S.serialize_state_with_nd_weights(96.0, w)
    cnt, flat = S.deserialize_as_image_1d_weights(st)
    assert cnt == 96.0 and flat.tobytes() == blob
    assert S.serialize_state_with_1d_weights(96.0, flat) == st
    S.nd_weights_to_arena(a, 0, back)
    assert torch.equal(a.state[0, :net.layout.n_master], a.state[1, :net.layout.n_master])


def test_hyperopt_batch_buckets_pack_configs():
    """with batch-size buckets TPE proposes only bucket values
    (inside the reference's [16, 256]), so a batch of 8 proposals falls into
    a few (model, batch) pack groups; 'none' keeps the full integer range."""
    import argparse
    from cerebro_ds_kpgi_amd.runners.common import hyperopt_grid
    from cerebro_ds_kpgi_amd.selection import hyperopt_helper as hh
    from cerebro_ds_kpgi_amd.utils.cli import get_main_parser
    # default: the reference space
    assert "batch_size_buckets" not in hyperopt_grid(get_main_parser().parse_args([]))
    args = get_main_parser().parse_args(["--hyperopt_models", "resnet50",
                                         "--hyperopt_batch_buckets", "16,32,64,128,256"])
    grid = hyperopt_grid(args)
    assert grid["batch_size_buckets"] == [16, 32, 64, 128, 256]
    hp, msts, trials, domain, rand, _ = hh.init_hyperopt(grid, argparse.Namespace(size=8))
    for i, m in enumerate(msts):
        trials.report(hp[i]["tid"], float(i))
    hp, msts, s, e = hh.hyperopt_add_one_batch_configs(None, hp, msts, domain, trials, 8,
                                                       rand=rand)
    assert all(m["batch_size"] in (16, 32, 64, 128, 256) for m in msts)
    assert len({(m["model"], m["batch_size"]) for m in msts[:8]}) <= 5
    args = get_main_parser().parse_args(["--hyperopt_batch_buckets", "none"])
    assert "batch_size_buckets" not in hyperopt_grid(args)
    assert len(hh.batch_choices(hyperopt_grid(args))) == 241
    with pytest.raises(ValueError):
        hh.batch_choices({"batch_size": [16, 256], "batch_size_buckets": [8]})
