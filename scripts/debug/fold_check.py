"""Debug: BN apply folded into the consumer conv vs the materialised path
(same kernels otherwise): dy of the first BN, its partial sums, grads."""
import torch
from cerebro_ds_kpgi_amd.ops import backend
from cerebro_ds_kpgi_amd.ops import nn as P
from cerebro_ds_kpgi_amd.runtime.arena import Arena, ModelLayout, ParamRef, ParamSpec

backend.set_backend("hip")
B, H, cin, c1, c2, G = 32, 14, 128, 128, 256, 8
specs = [ParamSpec("w1", (c1, 1, 1, cin), "weight", fan_in=cin),
         ParamSpec("g1", (c1,), "gamma"), ParamSpec("b1", (c1,), "beta"),
         ParamSpec("rm1", (c1,), "running_mean"), ParamSpec("rv1", (c1,), "running_var"),
         ParamSpec("w2", (c2, 3, 3, c1), "weight", fan_in=9 * c1),
         ParamSpec("g2", (c2,), "gamma"), ParamSpec("b2", (c2,), "beta"),
         ParamSpec("rm2", (c2,), "running_mean"), ParamSpec("rv2", (c2,), "running_var")]
L = ModelLayout(specs)
out = {}
for fold in (False, True, False):
    a = Arena(L, G, "cuda", torch.float32)
    for g in range(G):
        a.init_model(g, 11 + g)
    refs = {s.name: ParamRef(a, s) for s in specs}
    with torch.no_grad():
        torch.manual_seed(0)
        refs["g1"].master().uniform_(0.5, 1.5)
        refs["b1"].master().uniform_(-0.5, 0.5)
        a.sync_work()
    torch.manual_seed(4)
    x = torch.randn(B, H, H, G * cin, device="cuda").requires_grad_(True)
    h = P.conv_bn_act(x, refs["w1"], refs["g1"], refs["b1"], refs["rm1"], refs["rv1"], 1, 0,
                      True, None, 0.1, 1e-5, link_out=True, fold_out=fold)
    h.retain_grad()
    print("fold", fold, "tagged", getattr(h, "_cer_bnfold", None) is not None)
    y = P.conv_bn_act(h, refs["w2"], refs["g2"], refs["b2"], refs["rm2"], refs["rv2"], 1, 1,
                      True, None, 0.1, 1e-5)
    torch.manual_seed(5)
    gy = torch.randn_like(y)
    y.backward(gy)
    torch.cuda.synchronize()
    if fold in out:
        out["first_" + str(fold)] = out[fold]
    out[fold] = {"y": y.detach(), "dh": h.grad.detach(), "dx": x.grad.detach(),
                 "dW1": refs["w1"].grad().clone(), "dW2": refs["w2"].grad().clone(),
                 "dg1": refs["g1"].grad().clone(), "db1": refs["b1"].grad().clone(),
                 "dg2": refs["g2"].grad().clone()}
for k in out[False]:
    a, b = out[False][k].double(), out[True][k].double()
    f0 = out["first_False"][k].double()
    print(k, "first vs second materialised %.2e" % ((a - f0).norm() / a.norm()).item())
    print(k, "rel L2 fold vs materialised %.2e" % ((a - b).norm() / a.norm()).item())

# fp64 reference of dh (gradient w.r.t. the first unit's output y1) and dW2
import torch.nn.functional as F


def nchw(t):
    return t.permute(0, 3, 1, 2)


for fold in (False, True):
    pass
a = Arena(L, G, "cuda", torch.float32)
for g in range(G):
    a.init_model(g, 11 + g)
refs = {s.name: ParamRef(a, s) for s in specs}
with torch.no_grad():
    torch.manual_seed(0)
    refs["g1"].master().uniform_(0.5, 1.5)
    refs["b1"].master().uniform_(-0.5, 0.5)
torch.manual_seed(4)
x = torch.randn(B, H, H, G * cin, device="cuda")


def w64(name, cout, k, ci):
    return refs[name].master().double().view(G, cout, k, k, ci).permute(0, 1, 4, 2, 3).reshape(
        G * cout, ci, k, k)


def bn64(z, g, b):
    mean = z.mean((0, 2, 3))
    var = z.var((0, 2, 3), unbiased=False)
    return (z - mean.view(1, -1, 1, 1)) / torch.sqrt(var.view(1, -1, 1, 1) + 1e-5) * \
        g.view(1, -1, 1, 1) + b.view(1, -1, 1, 1)


x64 = nchw(x.double())
W1 = w64("w1", c1, 1, cin)
W2 = w64("w2", c2, 3, c1).requires_grad_(True)
y1 = torch.relu(bn64(F.conv2d(x64, W1, None, 1, 0, 1, G), refs["g1"].master().double().reshape(-1),
                     refs["b1"].master().double().reshape(-1))).detach().requires_grad_(True)
o2 = bn64(F.conv2d(y1, W2, None, 1, 1, 1, G), refs["g2"].master().double().reshape(-1),
          refs["b2"].master().double().reshape(-1))
o2 = o2 * nchw((out[True]["y"] > 0).double())
torch.manual_seed(5)
gy = torch.randn_like(out[True]["y"])
o2.backward(nchw(gy.double()))
dh64 = y1.grad.permute(0, 2, 3, 1)
dW2_64 = W2.grad.view(G, c2, c1, 3, 3).permute(0, 1, 3, 4, 2)
for fold in (False, True):
    print("fold", fold, "dh vs fp64 %.2e" % ((out[fold]["dh"].double() - dh64).norm() /
                                            dh64.norm()).item(),
          "dW2 vs fp64 %.2e" % ((out[fold]["dW2"].double().view(G, c2, 3, 3, c1) - dW2_64).norm()
                                / dW2_64.norm()).item())
