"""Uniform-K fp32 GEMM kernels and the HL weight image (GPU box).

Round 6: the fp32 fwd / dgrad kernels address 1x1 /
linear GEMMs (GM_GEMM) and k x k convs with 32-aligned channels (GM_TAP)
with wave-uniform per-step offsets, the 1x1 weight gradient runs as a plain
GEMM, and the optimizer keeps an HL image of the weights that the kernels
read without splitting (``runtime/arena.py`` ``Arena.whl``, conv.hip
``cer_conv_set_whl``).  The operands the MFMAs see are the same bits as
before, in the same K order, so with a pinned kernel variant the outputs
are bitwise equal to the im2col kernels' (``CER_UK=0``) with and without the
weight image; every new path is also checked against fp64.
"""

import pytest
import torch
import torch.nn.functional as F

from cerebro_ds_kpgi_amd.ops import backend
from cerebro_ds_kpgi_amd.ops import nn as P
from cerebro_ds_kpgi_amd.runtime.arena import Arena, ModelLayout, ParamRef, ParamSpec

pytestmark = pytest.mark.gpu

TOL = 1e-4

CASES = [
    # (B, H, W, Cin, Cout, k, stride, pad, G): ResNet-50 @112 shapes
    (32, 28, 28, 64, 64, 3, 1, 1, 8),       # GM_TAP fwd / dgrad
    (32, 14, 14, 128, 512, 1, 1, 0, 8),     # GM_GEMM all three ops
    (32, 28, 28, 256, 128, 1, 2, 0, 8),     # strided 1x1: GM_GEMM fwd + 1x1-geometry dgrad
    (32, 7, 7, 256, 256, 3, 1, 1, 2),
    (32, 4, 4, 2048, 512, 1, 1, 0, 1),      # one config: split-K
    (8, 14, 14, 64, 128, 3, 2, 1, 2),       # strided 3x3: GM_TAP fwd, GM_DGS dgrad (no UK)
    (4, 6, 6, 96, 32, 3, 1, 1, 2),          # 96 channels: 3 K steps per tap
    (2, 9, 11, 24, 40, 3, 2, 1, 2),         # unaligned: the im2col / generic paths
]


@pytest.fixture(autouse=True)
def _hip_backend():
    backend.set_backend("hip")
    backend.force_torch_ops([])
    backend.take_fallbacks()
    yield
    assert not backend.take_fallbacks(), "an op fell back to the PyTorch path"
    from cerebro_ds_kpgi_amd.ops import _hip
    _hip.lib().cer_conv_set_uk(1)
    _hip.conv_set_variant(0, -1)
    _hip.conv_set_variant(1, -1)


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def _arena(spec, G, whl):
    a = Arena(ModelLayout([spec]), G, "cuda", torch.float32)
    for g in range(G):
        a.init_model(g, 7 + g)
    if whl:
        assert a.enable_whl()
    return a, ParamRef(a, spec)


def _run(case, whl, uk, v=None):
    from cerebro_ds_kpgi_amd.ops import _hip
    B, H, W, cin, cout, k, s, p, G = case
    spec = ParamSpec("w", (cout, k, k, cin), "weight", fan_in=k * k * cin)
    a, ref = _arena(spec, G, whl)
    _hip.lib().cer_conv_set_uk(1 if uk else 0)
    if v is not None:
        _hip.conv_set_variant(0, v)
        _hip.conv_set_variant(1, v)
    torch.manual_seed(1)
    x = torch.randn(B, H, W, G * cin, device="cuda").requires_grad_(True)
    y = P.conv2d(x, ref, s, p)
    torch.manual_seed(3)
    gy = torch.randn_like(y)
    y.backward(gy)
    torch.cuda.synchronize()
    return a, ref, x, y.detach(), gy, x.grad.detach(), a.grad.clone()


@pytest.mark.parametrize("v", [0, 1, 2, 3, 5, 12, 13, 14, 15, 17, 24, 26])
@pytest.mark.parametrize("case", CASES)
def test_uk_bitwise_equals_im2col(case, v):
    """Pinned variant (no split-K): y and dx of the uniform-K kernels, with
    and without the HL weight image, equal the im2col kernels' bit for bit;
    dW (split-K atomics: order-dependent) to 1e-6."""
    base = _run(case, whl=False, uk=False, v=v)
    for whl in (False, True):
        got = _run(case, whl=whl, uk=True, v=v)
        assert torch.equal(got[3], base[3]), (case, v, whl, _rel(got[3], base[3]))
        assert torch.equal(got[5], base[5]), (case, v, whl, _rel(got[5], base[5]))
        assert _rel(got[6], base[6]) < 1e-6, (case, v, whl)


@pytest.mark.parametrize("case", CASES)
def test_uk_whl_fp32_vs_fp64(case):
    """Autotuned variants (split-K included), UK + HL weight image, vs fp64."""
    B, H, W, cin, cout, k, s, p, G = case
    a, ref, x, y, gy, dx, dw = _run(case, whl=True, uk=True)
    x64 = x.detach().double().permute(0, 3, 1, 2).requires_grad_(True)
    w64 = ref.master().double().permute(0, 1, 4, 2, 3).reshape(G * cout, cin, k, k)
    w64 = w64.clone().requires_grad_(True)
    y64 = F.conv2d(x64, w64, None, s, p, 1, G)
    y64.backward(gy.double().permute(0, 3, 1, 2))
    dw64 = w64.grad.view(G, cout, cin, k, k).permute(0, 1, 3, 4, 2).reshape(G, -1)
    e = (_rel(y, y64.detach().permute(0, 2, 3, 1)), _rel(dx, x64.grad.permute(0, 2, 3, 1)),
         _rel(dw.view(G, -1)[:, :dw64.shape[1]], dw64))
    print("uk+whl", case, "rel err y/dx/dw = %.2e %.2e %.2e" % e)
    assert max(e) < TOL, e


def test_linear_uk_whl_fp32_vs_fp64():
    """Linear layers (GM_GEMM on the 1x1 image) with the HL weight image."""
    G, B, K, N = 4, 32, 2048, 1000
    spec = ParamSpec("w", (N, K), "weight", fan_in=K)
    bspec = ParamSpec("b", (N,), "bias")
    a = Arena(ModelLayout([spec, bspec]), G, "cuda", torch.float32)
    for g in range(G):
        a.init_model(g, 3 + g)
    assert a.enable_whl()
    w, b = ParamRef(a, spec), ParamRef(a, bspec)
    torch.manual_seed(4)
    x = torch.randn(B, G * K, device="cuda").requires_grad_(True)
    y = P.linear(x, w, b, relu=False)
    gy = torch.randn_like(y)
    y.backward(gy)
    torch.cuda.synchronize()
    x64 = x.detach().double().view(B, G, K)
    W64 = w.master().double()                                   # [G, N, K]
    y64 = torch.einsum("bgk,gnk->bgn", x64, W64) + b.master().double().view(1, G, N)
    dx64 = torch.einsum("bgn,gnk->bgk", gy.double().view(B, G, N), W64)
    e = (_rel(y.view(B, G, N), y64), _rel(x.grad.view(B, G, K), dx64))
    print("linear uk+whl rel err y/dx = %.2e %.2e" % e)
    assert max(e) < TOL, e


def test_optimizer_writes_hl_image():
    """Adam and SGD write the HL image of the updated params (bit-equal to
    the HL image kernel over them); sync_work refreshes it after a host
    write; the image's fp32 value (hi + lo) is within bf16^2 of the params."""
    from cerebro_ds_kpgi_amd.ops import _hip
    from cerebro_ds_kpgi_amd.ops.optim import optimizer_step
    spec = ParamSpec("w", (64, 3, 3, 32), "weight", fan_in=288)
    for opt in ("adam", "sgd"):
        a = Arena(ModelLayout([spec]), 3, "cuda", torch.float32)
        for g in range(3):
            a.init_model(g, g)
            a.set_hparams(g, 1e-3, 1e-4)
        assert a.enable_whl()
        a.grad.normal_()
        a.grad_clean = True
        optimizer_step(a, opt)
        torch.cuda.synchronize()
        ref = torch.empty_like(a.whl)
        _hip.hl_image(a.params, ref)
        assert torch.equal(a.whl, ref), opt
        v = _hip.hl_to_fp32(a.whl)
        assert _rel(v, a.params) < 1e-5
        with torch.no_grad():
            a.params.mul_(0.5)
        a.sync_work()
        _hip.hl_image(a.params, ref)
        assert torch.equal(a.whl, ref)
