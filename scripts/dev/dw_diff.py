"""Depthwise fused-vs-plain forward difference probe: y of the plain 3x3
forward (cer_dwconv_fwd) against the forward + BN statistics kernel
(cer_dwconv_fwd_stats), and both against an fp64 oracle.  Prints, per case,
the number of differing elements, how many of them are signed-zero pairs,
the max |diff| and each kernel's max error against fp64.

    CER_HIP_LIB=libcerebro_hip_dwb.so python scripts/dev/dw_diff.py
"""

import torch
import torch.nn.functional as F

from cerebro_ds_kpgi_amd.ops import _hip
from cerebro_ds_kpgi_amd.runtime.arena import Arena, ModelLayout, ParamRef, ParamSpec


def case(G, C, B, H, s, pad):
    specs = [ParamSpec("dw", (C, 3, 3), "weight", fan_in=9)]
    a = Arena(ModelLayout(specs), G, "cuda", torch.float32)
    for g in range(G):
        a.init_model(g, 7 + g)
    a.sync_work()
    w = ParamRef(a, specs[0])
    torch.manual_seed(11)
    x = torch.randn(B, H, H + 1, G * C, device="cuda")
    y0 = _hip.dwconv_fwd(x, w, s, pad)
    y1 = _hip.dwconv_fwd_stats(x, w, s, pad)[0]
    torch.cuda.synchronize()
    pt, pb, pl, pr = _hip._pad4(pad)
    wt = torch.stack([a.master_view(specs[0])[g] for g in range(G)]).reshape(G * C, 1, 3, 3)
    xr = F.pad(x.double().permute(0, 3, 1, 2), (pl, pr, pt, pb))
    ref = F.conv2d(xr, wt.double(), stride=s, groups=G * C).permute(0, 2, 3, 1)
    ne = (y0 != y1)
    both_zero = ne & (y0 == 0) & (y1 == 0)
    d = (y0 - y1).abs().max().item()
    e0 = (y0.double() - ref).abs().max().item()
    e1 = (y1.double() - ref).abs().max().item()
    print("G=%d C=%d B=%d H=%d s=%d pad=%s: differ %d (signed zeros %d), max|y0-y1| %.3e, "
          "plain err %.3e, fused err %.3e" % (G, C, B, H, s, pad, int(ne.sum()), int(both_zero.sum()),
                                              d, e0, e1))
    if int(ne.sum()):
        idx = ne.nonzero()[:5].tolist()
        for i in idx:
            print("   at", i, y0[tuple(i)].item(), y1[tuple(i)].item(), ref[tuple(i)].item())


def main():
    for args in [(8, 96, 4, 14, 1, 1), (2, 512, 2, 9, 2, 1), (1, 144, 3, 11, 2, 1),
                 (1, 32, 8, 28, 1, 1), (2, 144, 3, 14, 2, (0, 1, 0, 1))]:
        case(*args)


if __name__ == "__main__":
    main()
