"""HIP kernel numerics vs the PyTorch fp32 oracle of the same op (GPU box)."""

import math

import pytest
import torch

from cerebro_ds_kpgi_amd.ops import backend

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _hip_backend():
    backend.set_backend("hip")
    backend.force_torch_ops([])
    yield
    backend.force_torch_ops([])


def _arena(G=3, model="tinycnn", dtype=torch.bfloat16, seed=0):
    from cerebro_ds_kpgi_amd.models import create_model_from_mst
    from cerebro_ds_kpgi_amd.runtime import Arena
    net = create_model_from_mst({"model": model})
    a = Arena(net.layout, G, "cuda", dtype)
    for g in range(G):
        a.init_model(g, seed + g)
        a.set_hparams(g, [1e-3, 3e-4, 1e-2][g % 3], [1e-4, 0.0, 1e-3][g % 3])
    return net, a


def test_adam_matches_torch():
    from cerebro_ds_kpgi_amd.ops.optim import adam_step
    net, a = _arena()
    net2, b = _arena()
    torch.manual_seed(0)
    for it in range(3):
        gr = torch.randn_like(a.grad)
        a.grad.copy_(gr)
        b.grad.copy_(gr)
        adam_step(a)                          # HIP
        backend.force_torch_ops(["adam"])
        adam_step(b)                          # oracle
        backend.force_torch_ops([])
    torch.cuda.synchronize()
    assert torch.allclose(a.state, b.state, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(a.work.float(), b.work.float(), rtol=1e-2, atol=1e-3)


@pytest.mark.parametrize("clean", [False, True])
def test_sgd_matches_torch(clean):
    from cerebro_ds_kpgi_amd.ops.optim import sgd_step
    net, a = _arena()
    net2, b = _arena()
    a.grad_clean = b.grad_clean = clean
    torch.manual_seed(0)
    for it in range(3):
        gr = torch.randn_like(a.grad)
        a.grad.copy_(gr)
        b.grad.copy_(gr)
        sgd_step(a)                           # HIP
        backend.force_torch_ops(["adam"])
        sgd_step(b)                           # oracle
        backend.force_torch_ops([])
    torch.cuda.synchronize()
    assert torch.allclose(a.state, b.state, rtol=1e-5, atol=1e-6)
    assert bool((a.grad == 0).all()) == clean


@pytest.mark.parametrize("N,G,B,dt", [(1000, 8, 32, torch.bfloat16), (1000, 8, 32, torch.float32),
                                      (2, 4, 64, torch.float32), (10, 3, 8, torch.bfloat16)])
def test_softmax_ce_matches_torch(N, G, B, dt):
    from cerebro_ds_kpgi_amd.ops.loss import softmax_ce
    torch.manual_seed(1)
    z = (3 * torch.randn(B, G * N, device="cuda")).to(dt)
    y = torch.randint(0, N, (G, B), device="cuda", dtype=torch.int32)
    acc1 = torch.zeros(G, 4, device="cuda")
    acc2 = torch.zeros(G, 4, device="cuda")
    z1 = z.clone().requires_grad_(True)
    z2 = z.clone().requires_grad_(True)
    l1 = softmax_ce(z1, y, acc1, G)
    (l1 * torch.arange(1, G + 1, device="cuda")).sum().backward()
    backend.force_torch_ops(["loss"])
    l2 = softmax_ce(z2, y, acc2, G)
    (l2 * torch.arange(1, G + 1, device="cuda")).sum().backward()
    torch.testing.assert_close(l1, l2, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(acc1[:, 0], acc2[:, 0], rtol=1e-4, atol=1e-3)
    # top-k counts: exact for fp32; bf16 logits can tie (tie order is arbitrary)
    tol = 0 if dt == torch.float32 else 1
    assert (acc1[:, 1:] - acc2[:, 1:]).abs().max().item() <= tol
    torch.testing.assert_close(z1.grad.float(), z2.grad.float(), rtol=2e-2, atol=2e-4)


def test_gather_matches_torch():
    from cerebro_ds_kpgi_amd.data.store import PartitionStore, gather_batch, input_buffers
    st = PartitionStore("imagenet", [0, 1, 2], 256, 64, "cuda")
    st.new_epoch(1)
    G, B = 3, 32
    part = torch.tensor([2, 0, 1], dtype=torch.int32, device="cuda")
    cur = torch.tensor([3], dtype=torch.int32, device="cuda")
    x1, y1 = input_buffers(st, G, B, torch.bfloat16)
    x2, y2 = input_buffers(st, G, B, torch.bfloat16)
    gather_batch(st, True, part, cur, B, x1, y1)
    backend.force_torch_ops(["gather"])
    gather_batch(st, True, part, cur, B, x2, y2)
    assert torch.equal(y1, y2)
    torch.testing.assert_close(x1.float(), x2.float(), rtol=1e-2, atol=1e-2)


def test_engine_one_round_on_gpu():
    from cerebro_ds_kpgi_amd.parallel import init_distributed
    from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine
    from cerebro_ds_kpgi_amd.selection import get_msts
    from cerebro_ds_kpgi_amd.config import catalog as cat
    msts = get_msts(cat.param_grid_tiny) * 2
    ctx = init_distributed()
    eng = MOPEngine(msts, ctx, EngineOptions(n_train=512, n_valid=64, slots_per_gpu=4,
                                             verbose=False, ckpt_every="none"))
    eng.run(2)
    for m, st in eng.mst_state.items():
        assert len(st["train_loss"]) == 2
        assert st["train_loss"][1] < st["train_loss"][0]
    eng.close()


@pytest.mark.parametrize("model,bs", [("confA", 32), ("mobilenetv2", 8), ("mobilenetv1", 8),
                                      ("vgg16", 8), ("densenet121", 8), ("resnext101", 4),
                                      ("resnet50_nobn", 8), ("resnet18", 8),
                                      ("nasnetmobile", 4), ("squeezenet", 8),
                                      ("densenet_tf1", 4)])
def test_engine_trains_model_family(model, bs):
    """Every model family steps through the HIP engine (graph capture included)."""
    from cerebro_ds_kpgi_amd.parallel import init_distributed
    from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine
    msts = [{"learning_rate": lr, "lambda_value": 1e-4, "batch_size": bs, "model": model}
            for lr in (1e-4, 1e-5)]
    eng = MOPEngine(msts, init_distributed(), EngineOptions(
        n_train=6 * bs, n_valid=2 * bs, slots_per_gpu=2, verbose=False, ckpt_every="none"))
    eng.run(1)
    for st in eng.mst_state.values():
        loss = st["train_loss"][0]
        assert len(st["train_loss"]) == 1 and math.isfinite(loss) and loss > 0.0
    eng.close()


@pytest.mark.parametrize("model,bs", [("resnet18", 8), ("mobilenetv2", 8), ("nasnetmobile", 4),
                                      ("resnet50", 4), ("vgg16", 4), ("densenet121", 4),
                                      ("mobilenetv1", 8), ("resnext101", 2),
                                      ("resnet50_nobn", 8), ("squeezenet", 8),
                                      ("densenet_tf1", 4), ("confA", 32)])
def test_graph_replay_matches_eager(model, bs):
    """HIP-graph replayed training (the default) follows the eager trajectory;
    a model whose step needs a PyTorch-path conv/pool stays eager instead."""
    from cerebro_ds_kpgi_amd.parallel import init_distributed
    from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine
    msts = [{"learning_rate": lr, "lambda_value": 1e-4, "batch_size": bs, "model": model}
            for lr in (1e-4, 1e-5)]
    losses = []
    for graphs in (False, True):
        eng = MOPEngine(msts, init_distributed(), EngineOptions(
            n_train=8 * bs, n_valid=2 * bs, slots_per_gpu=2, verbose=False, ckpt_every="none",
            use_graphs=graphs))
        eng.run(2)
        losses.append([st["train_loss"] + st["valid_loss"] for st in eng.mst_state.values()])
        if graphs:
            ws = [w for g in eng.groups.values() for w in g._work.values()]
            captured = any(w.graph is not None for w in ws)
            # every family but the ones with a PyTorch-path op (grouped conv of
            # ResNeXt, DenseNet's concat convs) must really replay a graph
            if model not in ("resnext101",):
                assert captured or all(w.eager_only for w in ws), model
            if model in ("resnet50", "resnet50_nobn", "vgg16", "confA", "resnet18",
                         "mobilenetv2", "nasnetmobile"):
                assert captured, "{}: no HIP graph was captured".format(model)
        eng.close()
    # every loss finite (train AND validation: the validation step is
    # graph-replayed too); the first round's training loss close — later
    # rounds of small-batch bf16 training drift apart chaotically (split-K
    # atomics are not bitwise deterministic), so they are only bounded
    for eager, graph in zip(*losses):
        assert all(math.isfinite(b) for b in graph), (eager, graph)
        assert abs(eager[0] - graph[0]) <= 3e-2 * abs(eager[0]), (eager, graph)
        for a, b in zip(eager, graph):
            assert abs(a - b) <= 0.6 * abs(a), (eager, graph)
