"""Locate the first non-finite activation of a NASNet train step (HIP vs oracle)."""
import torch
from cerebro_ds_kpgi_amd.models import create_model_from_mst
from cerebro_ds_kpgi_amd.ops import backend
from cerebro_ds_kpgi_amd.ops import nn as P
from cerebro_ds_kpgi_amd.ops.loss import softmax_ce
from cerebro_ds_kpgi_amd.runtime.arena import Arena

backend.set_backend("hip")
G, B = 2, 4
torch.manual_seed(0)
x = torch.randn(B, 112, 112, 3 * G, device="cuda").to(torch.bfloat16)
y = torch.randint(0, 1000, (G, B), device="cuda", dtype=torch.int32)

names = ["dwconv2d", "conv_bn_act", "bn_act", "conv2d", "avgpool2d", "maxpool2d", "cat_packed",
         "global_avgpool", "linear"]
first = []
for n in names:
    f = getattr(P, n)

    def wrap(*a, _f=f, _n=n, **k):
        out = _f(*a, **k)
        if not first and not torch.isfinite(out.float()).all():
            shapes = [tuple(t.shape) for t in a if isinstance(t, torch.Tensor)]
            fin = [bool(torch.isfinite(t.float()).all()) for t in a if isinstance(t, torch.Tensor)]
            first.append((_n, shapes, fin, tuple(out.shape)))
        return out
    setattr(P, n, wrap)

for force in ([], ["dwconv", "pool"], ["conv", "bn"], ["conv", "bn", "dwconv", "pool", "linear"]):
    backend.force_torch_ops(force)
    first.clear()
    net = create_model_from_mst({"model": "nasnetmobile"})
    a = Arena(net.layout, G, "cuda", torch.bfloat16)
    for g in range(G):
        a.init_model(g, 100 + g)
    net.bind(a)
    acc = torch.zeros(G, 4, device="cuda")
    out = net.forward(x, True)
    loss = softmax_ce(out, y, acc, G)
    loss.sum().backward()
    torch.cuda.synchronize()
    print("force", force, "loss", loss.tolist(), "grad finite", bool(torch.isfinite(a.grad).all()),
          "first non-finite:", first[:1])
