"""Engine-like step (fwd+bwd+Adam, grad_clean) captured in a HIP graph: loss per replay."""
import torch
from cerebro_ds_kpgi_amd.models import create_model_from_mst
from cerebro_ds_kpgi_amd.ops import backend
from cerebro_ds_kpgi_amd.ops.loss import softmax_ce
from cerebro_ds_kpgi_amd.ops.optim import adam_step
from cerebro_ds_kpgi_amd.runtime.arena import Arena

backend.set_backend("hip")
B = 4
for model in ("nasnetmobile", "mobilenetv2"):
  for G in (1, 2):
    for force in ([], ["conv", "bn", "dwconv", "pool", "linear"]):
        backend.force_torch_ops(force)
        torch.manual_seed(0)
        net = create_model_from_mst({"model": model})
        a = Arena(net.layout, G, "cuda", torch.bfloat16)
        a.grad_clean = True
        for g in range(G):
            a.init_model(g, 100 + g)
            a.set_hparams(g, 1e-5, 1e-4)
        net.bind(a)
        x = torch.randn(B, 112, 112, 3 * G, device="cuda").to(torch.bfloat16)
        y = torch.randint(0, 1000, (G, B), device="cuda", dtype=torch.int32)
        acc = torch.zeros(G, 4, device="cuda")
        out = {}

        def step():
            loss = softmax_ce(net.forward(x, True), y, acc, G)
            loss.sum().backward()
            out["gfin"] = torch.isfinite(a.grad).all()
            adam_step(a)
            out["loss"] = loss

        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        eager = []
        with torch.cuda.stream(s):
            for _ in range(3):
                step()
                eager.append(round(out["loss"][0].item(), 4))
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            step()
        res = []
        for _ in range(4):
            gr.replay()
            torch.cuda.synchronize()
            res.append((round(out["loss"][0].item(), 4), bool(out["gfin"]),
                        bool(torch.isfinite(a.params).all())))
        print(model, "G", G, "torch" if force else "hip", "eager", eager, "replays", res, flush=True)
        del gr
