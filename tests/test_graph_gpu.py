"""HIP-graph replay correctness (GPU box).

Round-1 symptom: replayed training steps went non-finite from the second
replay on (ResNet-50-noBN, captured validation, and -- found in round 2 -- the
bf16 ResNet-50 headline step itself, whose NaN early layers hid behind
finite losses because ReLU = fmaxf(x, 0) maps NaN to 0).  Root cause: a
``hipMemsetAsync`` captured into a HIP graph does not re-execute correctly
from the second replay on (ROCm 7.x, small fills; repro in
``scripts/debug/graph_memset_repro.py``).  Our launch paths now fill / copy
with kernels (``csrc/hip/common.h`` ``cer_zero_async``).  These tests pin it.
"""

import math

import pytest
import torch

from cerebro_ds_kpgi_amd.ops import backend, streams

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _hip_backend():
    backend.set_backend("hip")
    backend.force_torch_ops([])
    yield


@pytest.mark.parametrize("dtype,chunk", [(torch.float32, 0), (torch.bfloat16, 0),
                                         (torch.float32, "half")])
def test_fwd_bwd_graph_replays_equal_eager(dtype, chunk):
    """Captured fwd+bwd (no optimizer, fixed batch): every replay's gradient
    arena equals the eager one (same kernels, same variants).  "half": the
    split batch the runtime uses for packs of >= 4 configs (deferred_wgrad
    side_frac=0.5: the first half of the previous step's layers on the side
    stream, capped grid) -- a fork / join inside the captured graph; the
    eager gradient must also match the one-batch-at-the-end gradient."""
    _graph_replays(dtype, chunk)


def _graph_replays(dtype, chunk):
    from cerebro_ds_kpgi_amd.models import create_model_from_mst
    from cerebro_ds_kpgi_amd.ops.loss import softmax_ce
    from cerebro_ds_kpgi_amd.runtime import Arena
    G, B = 2, 8
    net = create_model_from_mst({"model": "resnet50"})
    a = Arena(net.layout, G, "cuda", dtype)
    for g in range(G):
        a.init_model(g, 2018 + g)
    net.bind(a)
    a.grad_clean = True
    torch.manual_seed(0)
    x = torch.randn(B, 112, 112, 3 * G, device="cuda").to(dtype)
    y = torch.randint(0, 1000, (G, B), device="cuda", dtype=torch.int32)
    acc = torch.zeros(G, 4, device="cuda")

    frac = [0.0]

    def step():
        a.grad.zero_()
        with streams.deferred_wgrad(True, side_frac=frac[0], key="graph_test"):
            softmax_ce(net.forward(x, True), y, acc, G).sum().backward()
        streams.join()
    m0 = a.master.clone()
    for _ in range(3):
        step()
    a.master.copy_(m0)
    step()
    torch.cuda.synchronize()
    ge = a.grad.clone()
    if chunk == "half":
        frac[0] = 0.5
    if chunk:
        for _ in range(2):
            a.master.copy_(m0)
            step()
        torch.cuda.synchronize()
        rel = ((a.grad.double() - ge.double()).norm() / ge.double().norm()).item()
        assert rel < 1e-3, rel
        ge = a.grad.clone()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        step()
    for r in range(4):
        a.master.copy_(m0)             # running statistics back to the same start
        graph.replay()
        torch.cuda.synchronize()
        assert torch.isfinite(a.grad).all(), r
        rel = ((a.grad.double() - ge.double()).norm() / ge.double().norm()).item()
        assert rel < 1e-3, (r, rel)    # split-K fp32 atomics: not bitwise


def test_kernel_fill_replays():
    """The fill/copy kernels that replace hipMemsetAsync replay correctly
    (bias-gradient workspace fill inside a captured bias+act backward)."""
    from cerebro_ds_kpgi_amd.ops import _hip
    from cerebro_ds_kpgi_amd.runtime.arena import Arena, ModelLayout, ParamRef, ParamSpec
    spec = ParamSpec("b", (24,), "bias")
    a = Arena(ModelLayout([spec]), 2, "cuda", torch.float32)
    ref = ParamRef(a, spec)
    dy = torch.randn(64, 48, device="cuda")
    yv = torch.randn(64, 48, device="cuda")
    _hip.bias_act_bwd(dy, yv, ref, 1)
    torch.cuda.synchronize()
    want = ref.grad().clone()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        _hip.bias_act_bwd(dy, yv, ref, 1)
    for _ in range(4):
        ref.grad().zero_()
        g.replay()
        torch.cuda.synchronize()
        torch.testing.assert_close(ref.grad(), want, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("model,dtype", [("resnet50", "bf16"), ("resnet50", "fp32"),
                                         ("resnet50_nobn", "fp32")])
def test_engine_many_replays_stay_finite(model, dtype):
    """30 replayed training steps keep every state row finite (the bf16
    headline step went non-finite at replay 2 before the fix)."""
    from cerebro_ds_kpgi_amd.parallel import init_distributed
    from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine
    bs = 8
    msts = [{"learning_rate": lr, "lambda_value": 1e-4, "batch_size": bs, "model": model}
            for lr in (1e-4, 1e-5)]
    eng = MOPEngine(msts, init_distributed(), EngineOptions(
        n_train=64 * bs, n_valid=2 * bs, slots_per_gpu=2, verbose=False, ckpt_every="none",
        compute_dtype=dtype, shuffle=False))
    eng.sched.start_epoch(1)
    eng.store.new_epoch(1)
    eng._hop_and_load(eng.sched.next_round())
    w = list(eng.groups.values())[0].current
    w.prepare(True)
    w.train_steps(30)
    torch.cuda.synchronize()
    assert w.graph is not None, "the step was not captured"
    assert torch.isfinite(w.arena.state).all()
    eng.close()


@pytest.mark.parametrize("model", ["resnet50", "resnet50_nobn"])
def test_captured_validation_matches_eager(model):
    """Graph-captured validation (now on by default) gives the eager
    validation metrics on the same weights, before and after an epoch
    boundary (the round-1 failure mode)."""
    from cerebro_ds_kpgi_amd.parallel import init_distributed
    from cerebro_ds_kpgi_amd.runtime import group as grp_mod
    from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine
    bs = 8
    msts = [{"learning_rate": lr, "lambda_value": 1e-4, "batch_size": bs, "model": model}
            for lr in (1e-4, 1e-5)]
    eng = MOPEngine(msts, init_distributed(), EngineOptions(
        n_train=8 * bs, n_valid=4 * bs, slots_per_gpu=2, verbose=False, ckpt_every="none",
        shuffle=False))
    saved = grp_mod._VALID_GRAPH
    try:
        for epoch in (1, 2):
            eng.sched.start_epoch(epoch)
            eng.store.new_epoch(epoch)
            eng._hop_and_load(eng.sched.next_round())
            w = list(eng.groups.values())[0].current
            w.prepare(True)
            w.train_steps(8)
            out = []
            for vg in (False, True, True):      # eager, capture + replay, replay
                grp_mod._VALID_GRAPH = vg
                w.vacc.zero_()
                w.validate(4)
                torch.cuda.synchronize()
                out.append(w.vacc.clone())
            assert w.vgraph is not None, "validation was not captured"
            for o in out[1:]:
                assert torch.isfinite(o).all()
                torch.testing.assert_close(o, out[0], rtol=1e-4, atol=1e-4)
            list(eng.groups.values())[0].end_round()
    finally:
        grp_mod._VALID_GRAPH = saved
        eng.close()


def test_side_split_at_every_layer_matches_one_batch():
    """the side wgrad batch must be ordered after BOTH streams of
    a block with a projection-shortcut branch.  Force the split after every
    possible layer count (so it fires on the branch stream for the shortcut
    layers, and on the main stream while a branch is open) and compare each
    step's gradient arena with the one-batch-at-the-end step, eagerly and
    replayed from a captured graph."""
    from cerebro_ds_kpgi_amd.models import create_model_from_mst
    from cerebro_ds_kpgi_amd.ops.loss import softmax_ce
    from cerebro_ds_kpgi_amd.runtime import Arena
    G, B = 4, 8
    net = create_model_from_mst({"model": "resnet50"})
    a = Arena(net.layout, G, "cuda", torch.float32)
    for g in range(G):
        a.init_model(g, 2018 + g)
    net.bind(a)
    a.grad_clean = True
    torch.manual_seed(0)
    x = torch.randn(B, 112, 112, 3 * G, device="cuda")
    y = torch.randint(0, 1000, (G, B), device="cuda", dtype=torch.int32)
    acc = torch.zeros(G, 4, device="cuda")
    frac = [0.0]

    def step():
        a.grad.zero_()
        with streams.deferred_wgrad(True, side_frac=frac[0], key="split_sweep"):
            softmax_ce(net.forward(x, True), y, acc, G).sum().backward()
        streams.join()

    m0 = a.master.clone()
    for _ in range(2):
        a.master.copy_(m0)
        step()
    torch.cuda.synchronize()
    ref = a.grad.double().clone()
    nlayers = streams._LAST["split_sweep"]
    assert nlayers > 40, nlayers
    frac[0] = 0.5
    try:
        for k in range(1, nlayers):
            streams._FORCE_SPLIT[0] = k
            a.master.copy_(m0)
            step()
            torch.cuda.synchronize()
            rel = ((a.grad.double() - ref).norm() / ref.norm()).item()
            assert rel < 1e-3, (k, rel)     # split-K fp32 atomics: not bitwise
        for k in range(1, nlayers, 5):
            streams._FORCE_SPLIT[0] = k
            a.master.copy_(m0)
            step()                           # the layer count of this split's key
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                step()
            for _ in range(2):
                a.master.copy_(m0)
                graph.replay()
                torch.cuda.synchronize()
                rel = ((a.grad.double() - ref).norm() / ref.norm()).item()
                assert rel < 1e-3, ("graph", k, rel)
            graph.reset()
    finally:
        streams._FORCE_SPLIT[0] = 0
