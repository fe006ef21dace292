"""Is a full-model grad mismatch a bug or bf16 chaos?  Compare HIP-bf16,
oracle-bf16, oracle-bf16 with a 1e-3 input perturbation, all against an
oracle fp32 run (GPU debug)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from cerebro_ds_kpgi_amd.ops import backend
from cerebro_ds_kpgi_amd.models import create_model_from_mst
from cerebro_ds_kpgi_amd.runtime import Arena
from cerebro_ds_kpgi_amd.ops.loss import softmax_ce

model = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4
G = 2
backend.set_backend("hip")
torch.manual_seed(11)
x32 = torch.randn(B, 112, 112, 3 * G, device="cuda")
y = torch.randint(0, 1000, (G, B), device="cuda", dtype=torch.int32)
ALL = ["conv", "bn", "pool", "bias", "linear", "loss", "adam", "gather"]


def run(force, dtype, x):
    backend.force_torch_ops(force)
    net = create_model_from_mst({"model": model})
    a = Arena(net.layout, G, "cuda", dtype)
    for g in range(G):
        a.init_model(g, 100 + g)
    net.bind(a)
    acc = torch.zeros(G, 4, device="cuda")
    loss = softmax_ce(net.forward(x.to(dtype), True), y, acc, G)
    loss.sum().backward()
    torch.cuda.synchronize()
    backend.force_torch_ops([])
    return loss.detach(), a.grad.clone()


ref_l, ref_g = run(ALL, torch.float32, x32)
cases = {
    "hip_bf16": run([], torch.bfloat16, x32),
    "oracle_bf16": run(ALL, torch.bfloat16, x32),
    "oracle_bf16_pert": run(ALL, torch.bfloat16, x32 * (1 + 1e-3 * torch.randn_like(x32))),
    "oracle_fp32_pert": run(ALL, torch.float32, x32 * (1 + 1e-3 * torch.randn_like(x32))),
}
print("fp32 loss", ref_l.tolist())
for k, (l, g) in cases.items():
    rel = ((g - ref_g).norm() / ref_g.norm()).item()
    print("%-18s loss %s  grad rel vs fp32 %.4f" % (k, [round(v, 4) for v in l.tolist()], rel))
