"""HL operand format (GPU box): conv-only activations and BN-backward
gradients stored as [8 x bf16 hi | 8 x bf16 lo] per 8 channels
(``csrc/hip/common.h`` st8_hl, ``conv.hip`` take_hi_lo, ``ops/_hip.py``).

The consumer convs of an HL tensor read exactly the (hi, lo) pair they would
have split from the fp32 value.  The claim is therefore bit-identity of
every deterministic result: with the conv kernel variants pinned, chained
units give the same outputs and input gradients bit for bit with the format
on and off.  The weight gradients agree to the rounding of their split-K
fp32 atomics, which accumulate in run-dependent order with or without HL.
A packed ResNet-50 trains the same through the engine.  The format itself
is checked against an independent torch split.
"""

import pytest
import torch

from cerebro_ds_kpgi_amd.ops import backend
from cerebro_ds_kpgi_amd.ops import nn as P
from cerebro_ds_kpgi_amd.runtime.arena import Arena, ModelLayout, ParamRef, ParamSpec

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _hip_backend():
    backend.set_backend("hip")
    backend.force_torch_ops([])
    backend.take_fallbacks()
    yield
    assert not backend.take_fallbacks(), "an op fell back to the PyTorch path"


def _hl(on):
    from cerebro_ds_kpgi_amd.ops import _hip
    _hip.HL_ENABLED = on


def _make(specs, G, seed=0):
    a = Arena(ModelLayout(specs), G, "cuda", torch.float32)
    torch.manual_seed(1000 + seed)
    for g in range(G):
        a.init_model(g, seed + g)
    for s in specs:
        if s.kind in ("gamma", "beta"):
            a.master_view(s).uniform_(0.5, 1.5)
        if s.kind == "running_var":
            a.master_view(s).uniform_(0.5, 2.0)
    a.sync_work()
    return a, {s.name: ParamRef(a, s) for s in specs}


def _torch_split(x):
    """(hi, lo) bf16 of fp32 x by round-to-nearest-even, as the kernels split."""
    hi = x.to(torch.bfloat16)
    lo = (x - hi.float()).to(torch.bfloat16)
    return hi, lo


def _chain(x, refs, hl_first):
    """unit 1 (its output HL when hl_first) -> unit 2 (3x3) -> unit 3 (1x1)."""
    h = P.conv_bn_act(x, refs["w1"], refs["g1"], refs["b1"], refs["rm1"], refs["rv1"], 1, 0, True,
                      None, 0.1, 1e-5, None, None, None, True, hl_first)
    h = P.conv_bn_act(h, refs["w2"], refs["g2"], refs["b2"], refs["rm2"], refs["rv2"], 1, 1, True,
                      None, 0.1, 1e-5, None, None, None, True, hl_first)
    return P.conv_bn_act(h, refs["w3"], refs["g3"], refs["b3"], refs["rm3"], refs["rv3"], 1, 0,
                         True, None, 0.1, 1e-5)


def _specs(cin, c1, c2, c3):
    out = []
    for i, (ci, co, k) in enumerate(((cin, c1, 1), (c1, c2, 3), (c2, c3, 1)), 1):
        out += [ParamSpec("w%d" % i, (co, k, k, ci), "weight", fan_in=k * k * ci),
                ParamSpec("g%d" % i, (co,), "gamma"), ParamSpec("b%d" % i, (co,), "beta"),
                ParamSpec("rm%d" % i, (co,), "running_mean"),
                ParamSpec("rv%d" % i, (co,), "running_var")]
    return out


def test_hl_bn_output_is_the_kernel_split():
    """A BN apply with HL output stores exactly torch's RNE (hi, lo) split of
    the fp32 output it would have written."""
    from cerebro_ds_kpgi_amd.ops import _hip
    specs = _specs(64, 64, 64, 256)
    G = 2
    x = torch.randn(4, 14, 14, G * 64, device="cuda")
    outs = []
    for on in (False, True):
        _hl(on)
        try:
            a, refs = _make(specs, G, seed=3)
            h = P.conv_bn_act(x, refs["w1"], refs["g1"], refs["b1"], refs["rm1"], refs["rv1"], 1,
                              0, True, None, 0.1, 1e-5, None, None, None, True, True)
            torch.cuda.synchronize()
            outs.append((h, _hip.is_hl(h)))
        finally:
            _hl(True)
    (y, f0), (yh, f1) = outs
    assert not f0 and f1, (f0, f1)
    hi, lo = _torch_split(y)
    C = y.shape[-1]
    words = yh.view(torch.int32).view(-1, C // 8, 2, 4)
    want_hi = hi.view(torch.int16).view(-1, C // 8, 8).view(torch.int32)
    want_lo = lo.view(torch.int16).view(-1, C // 8, 8).view(torch.int32)
    assert torch.equal(words[:, :, 0], want_hi.view(-1, C // 8, 4))
    assert torch.equal(words[:, :, 1], want_lo.view(-1, C // 8, 4))
    # and the fp32 view of the pair is hi + lo
    assert torch.equal(_hip.hl_to_fp32(yh), (hi.float() + lo.float()))


@pytest.mark.parametrize("G,B,H", [(2, 8, 14), (8, 4, 7)])
def test_hl_chain_bitwise_equals_fp32_chain(G, B, H):
    """Three chained training units (1x1 -> 3x3 -> 1x1, BN links on): with the
    first two outputs and every BN-backward gradient in HL format, the output,
    the input gradient and all parameter gradients are bit-identical to the
    all-fp32 run."""
    from cerebro_ds_kpgi_amd.ops import _hip
    specs = _specs(64, 64, 64, 256)
    torch.manual_seed(5)
    x0 = torch.randn(B, H, H, G * 64, device="cuda")
    gy = torch.randn(B, H, H, G * 256, device="cuda")
    res = []
    for on in (False, True):
        _hl(on)
        _hip.conv_set_variant(0, 0)          # same kernels in both runs (no split-K)
        _hip.conv_set_variant(1, 0)
        try:
            a, refs = _make(specs, G, seed=7)
            x = x0.clone().requires_grad_(True)
            y = _chain(x, refs, True)
            y.backward(gy)
            torch.cuda.synchronize()
            res.append((y.detach(), x.grad, a.grad.clone(), a.state.clone()))
        finally:
            _hl(True)
            _hip.conv_set_variant(0, -1)
            _hip.conv_set_variant(1, -1)
    for u, v, name in zip(res[0], res[1], ("y", "dx")):
        assert torch.equal(u, v), name
    assert torch.equal(res[0][3], res[1][3]), "running stats"
    g0, g1 = res[0][2].double(), res[1][2].double()
    rel = ((g0 - g1).norm() / g0.norm()).item()
    assert rel < 1e-6, rel
    assert _hip.HL_ENABLED


def test_resnet50_training_with_and_without_hl():
    """Packed ResNet-50 (2 configs, bs 4, fp32, HIP graphs, conv variants
    pinned): six engine training steps with the HL format land as close to
    the fp32-format run as two fp32-format runs land to each other (their
    only difference: the order of the split-K fp32 atomics, which Adam
    amplifies element-wise), and the HL run used HL conv launches."""
    from cerebro_ds_kpgi_amd.ops import _hip
    from cerebro_ds_kpgi_amd.parallel import init_distributed
    from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine
    bs = 4
    msts = [{"learning_rate": lr, "lambda_value": 1e-4, "batch_size": bs, "model": "resnet50"}
            for lr in (1e-3, 1e-4)]
    states = []
    for k in _hip.HL_COUNTS:
        _hip.HL_COUNTS[k] = 0
    for on in (False, False, True):
        _hl(on)
        _hip.conv_set_variant(0, 0)
        _hip.conv_set_variant(1, 0)
        try:
            eng = MOPEngine(msts, init_distributed(), EngineOptions(
                n_train=16 * bs, n_valid=2 * bs, slots_per_gpu=2, verbose=False,
                ckpt_every="none", compute_dtype="fp32", shuffle=False))
            eng.sched.start_epoch(1)
            eng.store.new_epoch(1)
            eng._hop_and_load(eng.sched.next_round())
            w = list(eng.groups.values())[0].current
            w.prepare(True)
            w.train_steps(6)
            torch.cuda.synchronize()
            assert w.graph is not None
            states.append(w.arena.state.clone())
            eng.close()
        finally:
            _hl(True)
            _hip.conv_set_variant(0, -1)
            _hip.conv_set_variant(1, -1)
    assert all(torch.isfinite(s).all() for s in states)

    def dist(a, b):
        na, nb = a.double().norm(dim=1), b.double().norm(dim=1)
        return ((na - nb).abs() / na).max().item()
    noise, hl = dist(states[0], states[1]), dist(states[0], states[2])
    print("per-config norm rel diff: fp32 vs fp32 %.2e, fp32 vs HL %.2e" % (noise, hl))
    # plain-vs-plain floor varies 5e-5 .. 1.5e-3 between boxes (atomics order)
    assert hl <= max(4 * noise, 2e-3), (hl, noise)
    assert min(_hip.HL_COUNTS.values()) > 0, _hip.HL_COUNTS
