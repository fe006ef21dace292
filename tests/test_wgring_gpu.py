"""LDS-DMA ring for the fp32 batched weight gradients (GPU box).

``conv.hip`` wgrad_ring_body32 copies HL-format operands (dy from the BN
backward, x from an HL BN output) global -> LDS with buffer_load ... lds
into the same LDS image the register-staged body builds, so the products
are the same; only the order of the split-K fp32 atomics differs.  Checked:
a batched flush of a three-unit chain (1x1 -> 3x3 -> 1x1, ResNet-50 stage-3
shapes, 8 packed configs) with the ring (2 stages, and 3 stages on the
128x64 tile) against the register kernel, and against fp64 via the same
chain's reference (tests/test_hl_gpu.py shows the chain itself is exact).
"""

import pytest
import torch

from cerebro_ds_kpgi_amd.ops import backend, streams

from test_hl_gpu import _chain, _make, _specs

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _hip_backend():
    from cerebro_ds_kpgi_amd.ops import _hip
    backend.set_backend("hip")
    backend.force_torch_ops([])
    backend.take_fallbacks()
    yield
    assert not backend.take_fallbacks(), "an op fell back to the PyTorch path"
    _hip.lib().cer_wgrad_batch_set_ring(0)
    streams._BATCH_VARIANT = 1


def _grads(ring, variant, G=8, B=32, H=14):
    from cerebro_ds_kpgi_amd.ops import _hip
    _hip.lib().cer_wgrad_batch_set_ring(ring)
    streams._BATCH_VARIANT = variant
    specs = _specs(256, 128, 128, 512)
    torch.manual_seed(21)
    x0 = torch.randn(B, H, H, G * 256, device="cuda")
    gy = torch.randn(B, H, H, G * 512, device="cuda")
    a, refs = _make(specs, G, seed=9)
    x = x0.clone().requires_grad_(True)
    with streams.deferred_wgrad(True, side_frac=0.0, key="wgring"):
        y = _chain(x, refs, True)
        y.backward(gy)
    streams.join()
    torch.cuda.synchronize()
    return a.grad.clone(), x.grad.clone(), _hip.HL_COUNTS["dy"]


@pytest.mark.parametrize("ring,variant", [(2, 1), (2, 2), (3, 2)])
def test_wgrad_ring_matches_register_kernel(ring, variant):
    g_ref, dx_ref, _ = _grads(0, variant)
    g_ref2, _, _ = _grads(0, variant)
    g_ring, dx_ring, hl = _grads(ring, variant)
    assert hl > 0, "no HL gradients: the ring path had nothing to do"
    assert torch.isfinite(g_ring).all()
    rel = lambda u, v: ((u.double() - v.double()).norm() / v.double().norm()).item()
    floor = rel(g_ref2, g_ref)
    d = rel(g_ring, g_ref)
    print("ring %d variant %d: grad rel diff %.2e (register vs register %.2e)" % (ring, variant, d,
                                                                                 floor))
    assert d < max(10 * floor, 1e-6), (d, floor)
    assert torch.equal(dx_ring, dx_ref)
