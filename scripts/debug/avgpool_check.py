"""Compare avgpool backward: HIP kernel vs torch (channels-last view, contiguous) vs CPU fp32."""
import torch
import torch.nn.functional as F
from cerebro_ds_kpgi_amd.ops import backend, nn as P

backend.set_backend("hip")
for (k, s, p, cip) in [(3, 1, 1, False), (2, 2, 0, False), (3, 2, 0, True)]:
    torch.manual_seed(0)
    x = torch.randn(2, 14, 14, 16, device="cuda").to(torch.bfloat16)
    g = None
    res = {}
    xx = x.clone().requires_grad_(True)
    y = P.avgpool2d(xx, k, s, p, count_include_pad=cip)
    g = torch.randn_like(y.float()).to(torch.bfloat16)
    y.backward(g)
    res["hip"] = xx.grad.float().cpu()
    xx = x.clone().requires_grad_(True)
    y2 = F.avg_pool2d(xx.permute(0, 3, 1, 2), k, s, p, count_include_pad=cip).permute(0, 2, 3, 1)
    y2.backward(g)
    res["torch_cl"] = xx.grad.float().cpu()
    xc = x.permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    y3 = F.avg_pool2d(xc, k, s, p, count_include_pad=cip)
    y3.backward(g.permute(0, 3, 1, 2).contiguous())
    res["torch_nchw"] = xc.grad.permute(0, 2, 3, 1).float().cpu()
    xf = x.float().cpu().permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    y4 = F.avg_pool2d(xf, k, s, p, count_include_pad=cip)
    y4.backward(g.float().cpu().permute(0, 3, 1, 2).contiguous())
    ref = xf.grad.permute(0, 2, 3, 1)
    print(k, s, p, cip, {n: round(((v - ref).norm() / ref.norm()).item(), 4) for n, v in res.items()},
          "fwd", round(((y.float().cpu() - y4.detach().permute(0, 2, 3, 1)).norm() / y4.norm()).item(), 4))
