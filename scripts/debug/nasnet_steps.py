"""NASNet multi-step training: per-step loss, eager vs HIP-graph replay."""
import torch
from cerebro_ds_kpgi_amd.models import create_model_from_mst
from cerebro_ds_kpgi_amd.ops import backend
from cerebro_ds_kpgi_amd.ops.loss import softmax_ce
from cerebro_ds_kpgi_amd.ops.optim import adam_step
from cerebro_ds_kpgi_amd.runtime.arena import Arena
from cerebro_ds_kpgi_amd.parallel import init_distributed
from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine

backend.set_backend("hip")
G, B = 2, 4
for force in ([], ["conv", "bn", "dwconv", "pool", "linear"]):
    backend.force_torch_ops(force)
    torch.manual_seed(0)
    net = create_model_from_mst({"model": "nasnetmobile"})
    a = Arena(net.layout, G, "cuda", torch.bfloat16)
    a.grad_clean = True
    for g in range(G):
        a.init_model(g, 100 + g)
        a.set_hparams(g, 1e-4, 1e-4)
    net.bind(a)
    losses = []
    for step in range(6):
        x = torch.randn(B, 112, 112, 3 * G, device="cuda").to(torch.bfloat16)
        y = torch.randint(0, 1000, (G, B), device="cuda", dtype=torch.int32)
        acc = torch.zeros(G, 4, device="cuda")
        loss = softmax_ce(net.forward(x, True), y, acc, G)
        loss.sum().backward()
        gfin = bool(torch.isfinite(a.grad).all())
        adam_step(a)
        losses.append((round(loss[0].item(), 3), gfin, bool(torch.isfinite(a.params).all()),
                       bool(torch.isfinite(a.state).all())))
    print("force", force, losses)
backend.force_torch_ops([])
for graphs in (False, True):
    msts = [{"learning_rate": lr, "lambda_value": 1e-4, "batch_size": 4, "model": "nasnetmobile"}
            for lr in (1e-4, 1e-5)]
    eng = MOPEngine(msts, init_distributed(), EngineOptions(
        n_train=24, n_valid=8, slots_per_gpu=2, verbose=False, ckpt_every="none",
        use_graphs=graphs))
    eng.run(1)
    print("graphs", graphs, {m: (st["train_loss"], st["valid_loss"]) for m, st in eng.mst_state.items()})
    eng.close()
