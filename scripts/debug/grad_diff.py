"""Per-parameter gradient diff HIP vs oracle for a full packed model (GPU debug)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from cerebro_ds_kpgi_amd.ops import backend
from cerebro_ds_kpgi_amd.models import create_model_from_mst
from cerebro_ds_kpgi_amd.runtime import Arena
from cerebro_ds_kpgi_amd.ops.loss import softmax_ce

model = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
G, B = 2, 4
backend.set_backend("hip")
torch.manual_seed(11)
x = torch.randn(B, 112, 112, 3 * G, device="cuda").to(torch.bfloat16)
y = torch.randint(0, 1000, (G, B), device="cuda", dtype=torch.int32)
res = []
for force in ([], ["conv", "bn", "pool", "bias", "linear"]):
    backend.force_torch_ops(force)
    net = create_model_from_mst({"model": model})
    a = Arena(net.layout, G, "cuda", torch.bfloat16)
    for g in range(G):
        a.init_model(g, 100 + g)
    net.bind(a)
    acc = torch.zeros(G, 4, device="cuda")
    loss = softmax_ce(net.forward(x, True), y, acc, G)
    loss.sum().backward()
    torch.cuda.synchronize()
    res.append((loss.detach(), a, net))
print("loss", res[0][0].tolist(), res[1][0].tolist())
ah, at = res[0][1], res[1][1]
for s in res[0][2].layout.train_specs:
    gh, gt = ah.grad_view(s).float(), at.grad_view(s).float()
    rel = ((gh - gt).norm() / (gt.norm() + 1e-12)).item()
    flag = "  <<<<" if rel > 0.05 else ""
    print("%-40s %-22s rel %.4f  |t| %.3e%s" % (s.name, str(s.shape), rel, gt.norm().item(), flag))
