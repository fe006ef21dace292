"""Residual-join activation masks as bits (bn.hip YM_M, ops._hip mask_ok).

The forward apply of a BN with a residual writes its ReLU mask as one bit
per element; the backward (BN apply / partials, and the BN-link statistics
in the consumer conv's dgrad epilogue) reads the bits instead of the fp32
output y.  The decisions are the same bits, so with the conv kernel
variants pinned two identical bottleneck-style chains -- residual join,
then a consumer conv whose dgrad carries the BN link -- give bit-identical
outputs, input gradients and running statistics with the mask on and off;
the weight gradients agree to the rounding of their split-K fp32 atomics.
The mask itself equals (y > 0) of the fp32 output, bit for bit.
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


def _mask(on):
    from cerebro_ds_kpgi_amd.ops import _hip
    _hip.BITMASK_ENABLED = on


def _make(specs, G, seed=0):
    a = Arena(ModelLayout(specs), G, "cuda", torch.float32)
    torch.manual_seed(1000 + seed)
    for g in range(G):
        a.init_model(g, seed + g)
    for s in specs:
        if s.kind in ("gamma", "beta"):
            a.master_view(s).uniform_(0.5, 1.5)
    a.sync_work()
    return a, {s.name: ParamRef(a, s) for s in specs}


def _specs(C, W):
    out = []
    for i, (ci, co) in enumerate(((C, W), (W, C), (C, W)), 1):
        out += [ParamSpec("w%d" % i, (co, 1, 1, ci), "weight", fan_in=ci),
                ParamSpec("g%d" % i, (co,), "gamma"), ParamSpec("b%d" % i, (co,), "beta"),
                ParamSpec("rm%d" % i, (co,), "running_mean"),
                ParamSpec("rv%d" % i, (co,), "running_var")]
    return out


def _chain(x, r):
    """x -> unit 1 (1x1) -> unit 2 (1x1, + x, ReLU: the residual join, its
    output linked to unit 3) -> unit 3 (1x1) whose dgrad computes unit 2's
    BN-backward statistics in its epilogue (the mask read there), then unit
    2's own BN backward (the mask read again)."""
    h = P.conv_bn_act(x, r["w1"], r["g1"], r["b1"], r["rm1"], r["rv1"], 1, 0, True, None,
                      link_out=True)
    h = P.conv_bn_act(h, r["w2"], r["g2"], r["b2"], r["rm2"], r["rv2"], 1, 0, True, x,
                      link_out=True)
    o = P.conv_bn_act(h, r["w3"], r["g3"], r["b3"], r["rm3"], r["rv3"], 1, 0, True, None)
    return o, h


@pytest.mark.parametrize("G,B,H", [(2, 8, 14), (8, 4, 7)])
def test_bitmask_chain_bitwise_equals_y_mask(G, B, H):
    from cerebro_ds_kpgi_amd.ops import _hip
    C, W = 64, 128
    specs = _specs(C, W)
    torch.manual_seed(5)
    x0 = torch.randn(B, H, H, G * C, device="cuda")
    go = torch.randn(B, H, H, G * W, device="cuda")
    res = []
    for on in (False, True):
        _mask(on)
        _hip.conv_set_variant(0, 0)
        _hip.conv_set_variant(1, 0)
        try:
            a, refs = _make(specs, G, seed=3)
            x = x0.clone().requires_grad_(True)
            o, h = _chain(x, refs)
            if on:
                m = getattr(h, "_cer_mask", None)
                assert m is not None, "no mask written"
                bits = torch.stack([(m.long() >> i) & 1 for i in range(8)], dim=-1).reshape(h.shape)
                assert torch.equal(bits.bool(), h.detach() > 0)
            o.backward(go)
            torch.cuda.synchronize()
            res.append((o.detach(), x.grad, a.state.clone(), a.grad.clone()))
        finally:
            _mask(True)
            _hip.conv_set_variant(0, -1)
            _hip.conv_set_variant(1, -1)
    assert torch.equal(res[0][0], res[1][0]), "output"
    assert torch.equal(res[0][1], res[1][1]), "input gradient"
    assert torch.equal(res[0][2], res[1][2]), "state (running statistics)"
    g0, g1 = res[0][3].double(), res[1][3].double()
    assert ((g0 - g1).norm() / g0.norm()).item() < 1e-6
