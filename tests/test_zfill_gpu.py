"""Strided 1x1 fp32 dgrad without an addend: the epilogue writes the
off-grid zeros (conv.hip NTParams::zfill / zfill_siblings) instead of a fill
kernel before the launch.  dx must be exactly zero off the stride grid even
when its memory held NaNs, and match an fp64 reference on the grid."""

import pytest
import torch

from cerebro_ds_kpgi_amd.ops import backend
from cerebro_ds_kpgi_amd.ops import nn as P
from cerebro_ds_kpgi_amd.runtime.arena import Arena, ModelLayout, ParamRef, ParamSpec

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("variant", [-1, 0, 1, 2, 12, 24])
@pytest.mark.parametrize("case", [(4, 14, 14, 64, 128, 2, 2), (2, 7, 7, 256, 64, 2, 3),
                                  (2, 9, 8, 32, 16, 3, 2)])
def test_strided_dgrad_zero_fill_in_epilogue(case, variant):
    from cerebro_ds_kpgi_amd.ops import _hip
    backend.set_backend("hip")
    B, H, W, cin, cout, st, G = case
    spec = ParamSpec("w", (cout, 1, 1, cin), "weight", fan_in=cin)
    a = Arena(ModelLayout([spec]), G, "cuda", torch.float32)
    for g in range(G):
        a.init_model(g, 70 + g)
    a.sync_work()
    ref = ParamRef(a, spec)
    torch.manual_seed(2)
    x = torch.randn(B, H, W, G * cin, device="cuda").requires_grad_(True)
    _hip.conv_set_variant(1, variant)
    try:
        y = P.conv2d(x, ref, st, 0)
        gy = torch.randn_like(y)
        # poison the allocator's free blocks: dx must not rely on zeroed memory
        junk = torch.full((B, H, W, G * cin), float("nan"), device="cuda")
        del junk
        y.backward(gy)
        torch.cuda.synchronize()
    finally:
        _hip.conv_set_variant(1, -1)
    dx = x.grad
    grid = torch.zeros(H, W, dtype=torch.bool, device="cuda")
    grid[::st, ::st] = True
    assert torch.isfinite(dx).all()
    assert (dx[:, ~grid] == 0).all()
    # fp64 reference on the grid
    w = ref.master().double().view(G, cout, cin)
    gyd = gy.double().view(B, y.shape[1], y.shape[2], G, cout)
    ref_dx = torch.einsum("bhwgo,goi->bhwgi", gyd, w).reshape(B, y.shape[1], y.shape[2], G * cin)
    got = dx[:, ::st, ::st].double()
    rel = ((got - ref_dx).norm() / ref_dx.norm()).item()
    print("zfill", case, variant, rel)
    assert rel < 1e-4
