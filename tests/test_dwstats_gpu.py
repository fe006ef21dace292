"""Depthwise 3x3 forward with the BN statistics of its output
(dwconv.hip dw_fwd_stats_kernel, ops.nn.dwconv2d stats=True).

The fused kernel writes the same y as the plain forward (same per-pixel
arithmetic) plus (sum, sum^2) partials in the conv epilogue's fp64 slab
format; the BN that consumes y then skips its statistics pass.  Compared
against the same chain with stats=False (the BN's own statistics pass):
y bit for bit, the BN output / running statistics / gradients to the
rounding of the different summation order.  Covers a wide pack (channel
blocks of 32 / 64 groups), idle channel lanes (144 / 8 = 18 groups),
stride 2 and Wo not a multiple of 4.
"""

import pytest
import torch

from cerebro_ds_kpgi_amd.ops import backend
from cerebro_ds_kpgi_amd.ops import nn as P
from cerebro_ds_kpgi_amd.runtime.arena import Arena, ModelLayout, ParamRef, ParamSpec

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _fused_at_every_size():
    from cerebro_ds_kpgi_amd.ops import _hip
    old = _hip.DW_STATS_MIN
    _hip.DW_STATS_MIN = 0
    yield
    _hip.DW_STATS_MIN = old


@pytest.fixture(autouse=True)
def _hip_backend():
    backend.set_backend("hip")
    backend.force_torch_ops([])
    backend.take_fallbacks()
    yield
    assert not backend.take_fallbacks(), "an op fell back to the PyTorch path"


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("G,C,B,H,s,dtype", [
    (8, 96, 4, 14, 1, torch.float32), (2, 512, 2, 9, 2, torch.float32),
    (1, 144, 3, 11, 2, torch.float32), (1, 32, 8, 28, 1, torch.float32),
    (4, 96, 4, 14, 1, torch.bfloat16)])
def test_dwconv_stats_matches_bn_pass(G, C, B, H, s, dtype):
    specs = [ParamSpec("dw", (C, 3, 3), "weight", fan_in=9), ParamSpec("g", (C,), "gamma"),
             ParamSpec("b", (C,), "beta"), ParamSpec("rm", (C,), "running_mean"),
             ParamSpec("rv", (C,), "running_var")]
    torch.manual_seed(11)
    x0 = torch.randn(B, H, H + 1, G * C, device="cuda").to(dtype)
    res = []
    for stats in (False, True):
        torch.manual_seed(1000)
        a = Arena(ModelLayout(specs), G, "cuda", dtype)
        for g in range(G):
            a.init_model(g, 7 + g)
        for sp in specs:
            if sp.kind in ("gamma", "beta"):
                a.master_view(sp).uniform_(0.5, 1.5)
        a.sync_work()
        r = {sp.name: ParamRef(a, sp) for sp in specs}
        x = x0.clone().requires_grad_(True)
        h = P.dwconv2d(x, r["dw"], s, 1, stats=stats)
        assert (getattr(h, "_cer_part", None) is not None) == stats
        o = P.bn_act(h, r["g"], r["b"], r["rm"], r["rv"], True, relu=6)
        assert getattr(h, "_cer_part", None) is None, "partials not consumed"
        torch.manual_seed(3)
        o.backward(torch.randn_like(o.float()).to(dtype))
        torch.cuda.synchronize()
        res.append((h.detach(), o.detach(), x.grad, a.state.clone(), a.grad.clone()))
    (h0, o0, dx0, st0, g0), (h1, o1, dx1, st1, g1) = res
    assert torch.equal(h0, h1), "y"
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert _rel(o1, o0) < tol
    assert _rel(st1, st0) < 1e-5
    assert _rel(dx1, dx0) < tol
    assert _rel(g1, g0) < tol


@pytest.mark.parametrize("G,C,B,H,dtype", [(8, 96, 4, 14, torch.float32), (1, 144, 3, 11, torch.float32),
                                           (4, 96, 4, 14, torch.bfloat16)])
def test_standalone_bn_link_matches_own_pass(G, C, B, H, dtype, monkeypatch):
    """dwconv -> BN (link_out) -> 1x1 conv_bn (MobileNetV2's depthwise BN and
    projection): the projection's dgrad epilogue computes the BN backward
    partials; against the BN's own backward pass."""
    from cerebro_ds_kpgi_amd.ops import _hip
    Co = 64
    specs = [ParamSpec("dw", (C, 3, 3), "weight", fan_in=9)]
    for i, c in ((1, C), (2, Co)):
        specs += [ParamSpec("g%d" % i, (c,), "gamma"), ParamSpec("b%d" % i, (c,), "beta"),
                  ParamSpec("rm%d" % i, (c,), "running_mean"),
                  ParamSpec("rv%d" % i, (c,), "running_var")]
    specs.insert(5, ParamSpec("w2", (Co, 1, 1, C), "weight", fan_in=C))
    used = []
    real = _hip.bn_act_bwd

    def spy(*a, **k):
        used.append(k.get("part") is not None)
        return real(*a, **k)
    monkeypatch.setattr(_hip, "bn_act_bwd", spy)
    torch.manual_seed(12)
    x0 = torch.randn(B, H, H, G * C, device="cuda").to(dtype)
    go = torch.randn(B, H, H, G * Co, device="cuda").to(dtype)
    res = []
    for link in (False, True):
        used.clear()
        torch.manual_seed(1000)
        a = Arena(ModelLayout(specs), G, "cuda", dtype)
        for g in range(G):
            a.init_model(g, 5 + g)
        for sp in specs:
            if sp.kind in ("gamma", "beta"):
                a.master_view(sp).uniform_(0.5, 1.5)
        a.sync_work()
        r = {sp.name: ParamRef(a, sp) for sp in specs}
        _hip.conv_set_variant(0, 0)
        _hip.conv_set_variant(1, 0)
        try:
            x = x0.clone().requires_grad_(True)
            h = P.dwconv2d(x, r["dw"], 1, 1, stats=True)
            h = P.bn_act(h, r["g1"], r["b1"], r["rm1"], r["rv1"], True, relu=6, link_out=link)
            o = P.conv_bn_act(h, r["w2"], r["g2"], r["b2"], r["rm2"], r["rv2"], 1, 0, 6)
            o.backward(go)
            torch.cuda.synchronize()
        finally:
            _hip.conv_set_variant(0, -1)
            _hip.conv_set_variant(1, -1)
        # the depthwise BN is the last BN backward to run
        assert used[-1] == link, used
        res.append((o.detach(), x.grad, a.state.clone(), a.grad.clone()))
    (o0, dx0, st0, g0), (o1, dx1, st1, g1) = res
    assert torch.equal(o0, o1)
    assert torch.equal(st0, st1)
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert _rel(dx1, dx0) < tol
    assert _rel(g1, g0) < tol


@pytest.mark.parametrize("G,C,B,H,s,pad,dtype", [
    (8, 96, 4, 14, 1, 1, torch.float32), (2, 144, 3, 11, 2, 1, torch.float32),
    (2, 144, 3, 14, 2, (0, 1, 0, 1), torch.float32), (1, 64, 2, 9, 2, (0, 1, 0, 1), torch.float32),
    (4, 96, 4, 14, 2, 1, torch.bfloat16), (4, 96, 4, 14, 2, (0, 1, 0, 1), torch.bfloat16)])
def test_dwconv_dgrad_bn_link_matches_own_pass(G, C, B, H, s, pad, dtype, monkeypatch):
    """1x1 conv_bn (ReLU6, link_out) -> dwconv -> BN (MobileNetV2's expansion
    unit and depthwise conv): the depthwise dgrad computes the expansion BN's
    backward partials; against that BN's own backward pass.  Stride 2 with
    both left-pad parities (symmetric 1 and Keras correct_pad (0, 1)): the
    fused kernel's static dy column window depends on it."""
    from cerebro_ds_kpgi_amd.ops import _hip
    Ci = 32
    specs = [ParamSpec("w1", (C, 1, 1, Ci), "weight", fan_in=Ci)]
    for i in (1, 2):
        specs += [ParamSpec("g%d" % i, (C,), "gamma"), ParamSpec("b%d" % i, (C,), "beta"),
                  ParamSpec("rm%d" % i, (C,), "running_mean"),
                  ParamSpec("rv%d" % i, (C,), "running_var")]
        if i == 1:
            specs.append(ParamSpec("dw", (C, 3, 3), "weight", fan_in=9))
    used = []
    real = _hip.bn_act_bwd

    def spy(*a, **k):
        used.append(k.get("part") is not None)
        return real(*a, **k)
    monkeypatch.setattr(_hip, "bn_act_bwd", spy)
    torch.manual_seed(13)
    x0 = torch.randn(B, H, H, G * Ci, device="cuda").to(dtype)
    res = []
    for link in (False, True):
        used.clear()
        torch.manual_seed(1000)
        a = Arena(ModelLayout(specs), G, "cuda", dtype)
        for g in range(G):
            a.init_model(g, 9 + g)
        for sp in specs:
            if sp.kind in ("gamma", "beta"):
                a.master_view(sp).uniform_(0.5, 1.5)
        a.sync_work()
        r = {sp.name: ParamRef(a, sp) for sp in specs}
        _hip.conv_set_variant(0, 0)
        _hip.conv_set_variant(1, 0)
        try:
            x = x0.clone().requires_grad_(True)
            h = P.conv_bn_act(x, r["w1"], r["g1"], r["b1"], r["rm1"], r["rv1"], 1, 0, 6,
                              link_out=link)
            h = P.dwconv2d(h, r["dw"], s, pad, stats=True)
            o = P.bn_act(h, r["g2"], r["b2"], r["rm2"], r["rv2"], True, relu=6)
            torch.manual_seed(3)
            o.backward(torch.randn_like(o.float()).to(dtype))
            torch.cuda.synchronize()
        finally:
            _hip.conv_set_variant(0, -1)
            _hip.conv_set_variant(1, -1)
        assert used[-1] == link, used       # the expansion BN's backward runs last
        res.append((o.detach(), x.grad, a.state.clone(), a.grad.clone()))
    (o0, dx0, st0, g0), (o1, dx1, st1, g1) = res
    assert torch.equal(o0, o1)
    assert torch.equal(st0, st1)
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert _rel(dx1, dx0) < tol
    assert _rel(g1, g0) < tol
