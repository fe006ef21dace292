"""Projection-shortcut BN applied inside the block's last BN apply
(ops.nn.PendingBN, bn.hip ResBN / cer_bn_set_res_bn) on the GPU box.

The shortcut unit of a ResNet projection block returns its conv output; the
block's last apply computes act(BN(z) + BN_s(zs)) and writes the shortcut
BN's batch statistics and running statistics.  Same arithmetic as applying
the shortcut BN on its own and adding, so a training step must match the
non-deferred path to rounding."""

import pytest
import torch

from cerebro_ds_kpgi_amd.ops import backend
from cerebro_ds_kpgi_amd.ops import nn as P
from cerebro_ds_kpgi_amd.runtime.arena import Arena

pytestmark = pytest.mark.gpu


def _step(model, defer, G=2, B=4):
    from cerebro_ds_kpgi_amd.models import create_model_from_mst
    from cerebro_ds_kpgi_amd.models import resnet
    from cerebro_ds_kpgi_amd.ops.loss import softmax_ce
    backend.set_backend("hip")
    made = []
    orig = P.PendingBN.__init__

    def spy(self, *a, **k):
        made.append(1)
        orig(self, *a, **k)
    old = resnet._SC_DEFER
    resnet._SC_DEFER = defer
    P.PendingBN.__init__ = spy
    try:
        torch.manual_seed(11)
        x = torch.randn(B, 112, 112, 3 * G, device="cuda")
        y = torch.randint(0, 1000, (G, B), device="cuda", dtype=torch.int32)
        net = create_model_from_mst({"model": model})
        a = Arena(net.layout, G, "cuda", torch.float32)
        for g in range(G):
            a.init_model(g, 100 + g)
        a.grad_clean = True
        a.grad.zero_()
        net.bind(a)
        acc = torch.zeros(G, 4, device="cuda")
        loss = softmax_ce(net.forward(x, True), y, acc, G)
        loss.sum().backward()
        torch.cuda.synchronize()
    finally:
        resnet._SC_DEFER = old
        P.PendingBN.__init__ = orig
    return loss.detach(), a.grad.clone(), a.master.clone(), len(made)


@pytest.mark.parametrize("model", ["resnet50", "resnet18"])
def test_deferred_shortcut_bn_matches(model):
    l1, g1, m1, n1 = _step(model, True)
    l0, g0, m0, n0 = _step(model, False)
    d = ((g1.double() - g0.double()).norm() / g0.double().norm()).item()
    print(model, "deferred shortcut BNs", n1, "grad rel diff", d)
    assert n0 == 0 and n1 == (4 if model == "resnet50" else 3)
    # (losses to rounding: the fp64 BN-statistics atomics' order varies run to run)
    assert ((l1 - l0).abs() / l0.abs()).max().item() < 1e-6
    assert torch.isfinite(g1).all()
    assert d < 1e-5, d
    # running statistics (written by the consumer's apply) and the rest of the
    # arena rows: the parameters are untouched by a forward/backward, the
    # running mean / var of every BN layer updated once
    dm = ((m1.double() - m0.double()).abs().max()).item()
    assert dm < 1e-5, dm


def test_pending_bn_materialize():
    """A consumer that cannot fuse the deferred apply gets BN_s(zs) as a tensor."""
    from cerebro_ds_kpgi_amd.models import create_model_from_mst
    backend.set_backend("hip")
    G, B = 2, 4
    torch.manual_seed(3)
    net = create_model_from_mst({"model": "resnet50"})
    a = Arena(net.layout, G, "cuda", torch.float32)
    for g in range(G):
        a.init_model(g, 7 + g)
    net.bind(a)
    blk = net.blocks[0]
    x = torch.randn(B, 28, 28, 64 * G, device="cuda")
    ref = lambda p: net.ref(p)  # noqa: E731
    c, b = blk["cs"], blk["bs"]
    args = (x, ref(c.w), ref(b.g), ref(b.b), ref(b.rm), ref(b.rv), c.stride, c.pad, False)
    rm0, rv0 = ref(b.rm).master().clone(), ref(b.rv).master().clone()
    want = P.conv_bn_act(*args)
    rm1, rv1 = ref(b.rm).master().clone(), ref(b.rv).master().clone()
    ref(b.rm).master().copy_(rm0)
    ref(b.rv).master().copy_(rv0)
    got = P.conv_bn_act(*args, defer=True)
    pend = got._cer_pending_bn
    assert pend is not None and torch.equal(got, pend.z)
    y = pend.materialize()
    torch.cuda.synchronize()
    assert ((y - want).abs().max() / want.abs().max()).item() < 1e-6
    # the running statistics advanced once, as by the plain unit
    assert torch.allclose(ref(b.rm).master(), rm1, rtol=1e-6, atol=1e-7)
    assert torch.allclose(ref(b.rv).master(), rv1, rtol=1e-6, atol=1e-7)
    with pytest.raises(AssertionError):
        pend.claim()
