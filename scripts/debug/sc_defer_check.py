"""Deferred shortcut BN (ops.nn.PendingBN) vs the plain unit, forward only,
one ResNet-50 projection block: block output, the shortcut BN's batch
statistics and the running statistics, as max abs differences."""
import torch

from cerebro_ds_kpgi_amd.models import create_model_from_mst, resnet
from cerebro_ds_kpgi_amd.ops import backend
from cerebro_ds_kpgi_amd.ops import nn as P
from cerebro_ds_kpgi_amd.runtime.arena import Arena


def run(defer, G=2, B=4):
    backend.set_backend("hip")
    resnet._SC_DEFER = defer
    torch.manual_seed(5)
    net = create_model_from_mst({"model": "resnet50"})
    a = Arena(net.layout, G, "cuda", torch.float32)
    for g in range(G):
        a.init_model(g, 100 + g)
    net.bind(a)
    r = net.ref
    blk = net.blocks[0]
    x = torch.randn(B, 28, 28, 64 * G, device="cuda")
    mk = lambda c, b: (r(c.w), r(b.g), r(b.b), r(b.rm), r(b.rv), c.stride, c.pad)  # noqa: E731
    sc = P.conv_bn_act(x, *mk(blk["cs"], blk["bs"]), False, defer=defer)
    h = P.conv_bn_act(x, *mk(blk["c1"], blk["b1"]), True)
    h = P.conv_bn_act(h, *mk(blk["c2"], blk["b2"]), True)
    out = P.conv_bn_act(h, *mk(blk["c3"], blk["b3"]), True, residual=sc)
    torch.cuda.synchronize()
    return out, sc, a.master.clone()


o1, s1, m1 = run(True)
o0, s0, m0 = run(False)
print("out max abs diff", (o1 - o0).abs().max().item(), "max", o0.abs().max().item())
print("sc is pending:", getattr(s1, "_cer_pending_bn", None) is not None)
print("arena (running stats) max abs diff", (m1 - m0).abs().max().item())
o0b, _, m0b = run(False)
print("plain vs plain: out", (o0b - o0).abs().max().item(), "arena", (m0b - m0).abs().max().item())

import sys  # noqa: E402
sys.path.insert(0, "tests")
from test_sc_defer_gpu import _step  # noqa: E402
for a, b in ((False, False), (True, False), (True, True)):
    l1, g1, _, _ = _step("resnet50", a)
    l0, g0, _, _ = _step("resnet50", b)
    d = ((g1.double() - g0.double()).norm() / g0.double().norm()).item()
    print("step defer", a, "vs", b, "loss rel", ((l1 - l0).abs() / l0.abs()).max().item(),
          "grad rel", d)
