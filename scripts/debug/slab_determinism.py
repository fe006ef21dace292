"""Is the graph-vs-eager gradient gap with atomic BN slabs plain run-to-run
non-determinism (fp32 atomics' order, amplified through 50 BN layers)?
Two eager fwd+bwd from the same state, gradient arena compared."""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from cerebro_ds_kpgi_amd.models import create_model_from_mst  # noqa: E402
from cerebro_ds_kpgi_amd.ops import set_backend, streams  # noqa: E402
from cerebro_ds_kpgi_amd.ops.loss import softmax_ce  # noqa: E402
from cerebro_ds_kpgi_amd.runtime import Arena  # noqa: E402

set_backend("hip")
G, B = 2, 8
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
m0 = a.master.clone()


def step():
    a.master.copy_(m0)
    a.grad.zero_()
    with streams.deferred_wgrad(True, key="det"):
        softmax_ce(net.forward(x, True), y, acc, G).sum().backward()
    streams.join()
    torch.cuda.synchronize()
    return a.grad.clone(), a.master.clone()


for _ in range(3):
    step()
g1, s1 = step()
g2, s2 = step()
rel = ((g1.double() - g2.double()).norm() / g1.double().norm()).item()
rs = ((s1.double() - s2.double()).norm() / s1.double().norm()).item()
print("slabs={} eager-vs-eager grad rel {:.3e} state rel {:.3e}".format(
    os.environ.get("CER_BN_ATOMIC_SLABS", "2"), rel, rs))
