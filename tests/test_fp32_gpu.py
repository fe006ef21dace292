"""Reference-precision (fp32) HIP kernels vs fp64 references (GPU box).

The reference trains in fp32 (TF 1.14 / PyTorch 1.4 defaults,
``/root/reference/cerebro_gpdb/run_pytorchddp.py:285-309``).  Our fp32 mode
keeps every tensor fp32 in HBM and runs convolutions / linears as 3-pass
split-bf16 MFMA GEMMs with fp32 accumulation (``csrc/hip/conv.hip``).

Bound: relative L2 error vs an fp64 reference of the same op <= 1e-4
(``TOL``).  The 3-pass products carry ~2^-16 relative error each; measured
errors are ~1e-6 - 1e-5 (the printed ratios on the GPU box).  ReLU backward
is compared under the mask of OUR forward output: a pre-activation within
rounding of 0 may flip sign between fp32 and fp64, and a flipped fraction f
of the mask alone moves the relative L2 of every gradient by ~sqrt(f)
(~1e-3 at f ~ 1e-6) whatever the implementation.  Conv cases
include the real ResNet-50 layer shapes of the headline step (B = 32,
G = 8 packed configs).  Each test also checks that the fp32 HIP path ran
(no silent fallback to the PyTorch / MIOpen oracle).
"""

import pytest
import torch
import torch.nn.functional as F

from cerebro_ds_kpgi_amd.ops import backend
from cerebro_ds_kpgi_amd.ops import nn as P
from cerebro_ds_kpgi_amd.runtime.arena import Arena, ModelLayout, ParamRef, ParamSpec

pytestmark = pytest.mark.gpu

TOL = 1e-4


@pytest.fixture(autouse=True)
def _hip_backend():
    backend.set_backend("hip")
    backend.force_torch_ops([])
    backend.take_fallbacks()
    yield
    assert not backend.take_fallbacks(), "an op fell back to the PyTorch path"
    backend.force_torch_ops([])


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def _make(specs, G, seed=0):
    a = Arena(ModelLayout(specs), G, "cuda", torch.float32)
    torch.manual_seed(1000 + seed)
    for g in range(G):
        a.init_model(g, seed + g)
    for s in specs:
        if s.kind in ("gamma", "beta", "bias", "running_mean"):
            a.master_view(s).uniform_(-0.5, 1.5)
        if s.kind == "running_var":
            a.master_view(s).uniform_(0.5, 2.0)
    a.sync_work()
    return a, {s.name: ParamRef(a, s) for s in specs}


def _nchw(x):
    return x.permute(0, 3, 1, 2)


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def _w64(wref):
    """[G, cout, kh, kw, cin] arena weights -> fp64 [G*cout, cin, kh, kw]."""
    G = wref.G
    cout, kh, kw, cin = wref.spec.shape
    return wref.master().double().permute(0, 1, 4, 2, 3).reshape(G * cout, cin, kh, kw)


def _fp32_conv_ran():
    from cerebro_ds_kpgi_amd.ops import _hip
    return any("float32" in str(k[1][0]) for k in _hip.tuned_variants())


CONV_CASES = [
    # (B, H, W, Cin, Cout, k, stride, pad, G) -- ResNet-50 @112, B = 32, G = 8
    (32, 28, 28, 64, 64, 3, 1, 1, 8),
    (32, 28, 28, 256, 128, 1, 2, 0, 8),
    (32, 14, 14, 128, 512, 1, 1, 0, 8),
    (32, 7, 7, 256, 256, 3, 1, 1, 8),
    (32, 4, 4, 512, 512, 3, 1, 1, 8),
    (32, 7, 7, 1024, 2048, 1, 2, 0, 8),
    (32, 112, 112, 3, 64, 7, 2, 3, 8),     # stem (generic element gather in this op form)
    # one config (per-GPU work at N = 8): split-K paths
    (32, 4, 4, 512, 512, 3, 1, 1, 1),
    (32, 4, 4, 2048, 512, 1, 1, 0, 1),
    # unaligned / odd shapes (generic gather, transposed-weight dgrad fallback)
    (2, 9, 11, 24, 40, 3, 2, 1, 2),
    (3, 6, 5, 8, 12, 3, 1, 0, 3),
    (4, 14, 14, 64, 128, 3, 2, 1, 2),       # strided 3x3 dgrad
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fp32_vs_fp64(case):
    B, H, W, cin, cout, k, s, p, G = case
    spec = ParamSpec("w", (cout, k, k, cin), "weight", fan_in=k * k * cin)
    a, refs = _make([spec], G)
    torch.manual_seed(1)
    x = torch.randn(B, H, W, G * cin, device="cuda")
    xx = x.clone().requires_grad_(True)
    y = P.conv2d(xx, refs["w"], s, p)
    assert y.dtype == torch.float32
    torch.manual_seed(3)
    gy = torch.randn_like(y)
    y.backward(gy)
    torch.cuda.synchronize()
    # fp64 reference
    x64 = _nchw(x.double()).requires_grad_(True)
    w64 = _w64(refs["w"]).requires_grad_(True)
    y64 = F.conv2d(x64, w64, None, s, p, 1, G)
    y64.backward(_nchw(gy.double()))
    dw64 = w64.grad.view(G, cout, cin, k, k).permute(0, 1, 3, 4, 2)
    e = (_rel(y, _nhwc(y64.detach())), _rel(xx.grad, _nhwc(x64.grad)),
         _rel(a.grad.view(G, -1)[:, :dw64[0].numel()], dw64.reshape(G, -1)))
    print("conv", case, "rel err y/dx/dw = %.2e %.2e %.2e" % e)
    assert max(e) < TOL, e
    assert _fp32_conv_ran()


@pytest.mark.parametrize("v", [3, 4, 5, 9, 10, 11])
@pytest.mark.parametrize("case", [CONV_CASES[0], CONV_CASES[1], CONV_CASES[2], CONV_CASES[5],
                                  CONV_CASES[7], (2, 9, 11, 32, 40, 3, 2, 1, 2)])
def test_conv_fwd_lds_ring_fp32_vs_fp64(case, v):
    """The fp32 LDS-DMA ring forward kernels (pipe_nt32, every tile shape,
    with and without split-K), pinned, vs an fp64 conv."""
    from cerebro_ds_kpgi_amd.ops import _hip
    B, H, W, cin, cout, k, s, p, G = case
    spec = ParamSpec("w", (cout, k, k, cin), "weight", fan_in=k * k * cin)
    a, refs = _make([spec], G)
    torch.manual_seed(1)
    x = torch.randn(B, H, W, G * cin, device="cuda")
    _hip.conv_set_variant(0, v)
    try:
        y = P.conv2d(x, refs["w"], s, p)
        torch.cuda.synchronize()
    finally:
        _hip.conv_set_variant(0, -1)
    y64 = F.conv2d(_nchw(x.double()), _w64(refs["w"]), None, s, p, 1, G)
    e = _rel(y, _nhwc(y64))
    print("ring fwd", case, v, "rel err %.2e" % e)
    assert e < TOL, e


@pytest.mark.parametrize("v", list(range(12, 24)))
@pytest.mark.parametrize("case", [CONV_CASES[0], CONV_CASES[1], CONV_CASES[2], CONV_CASES[5],
                                  CONV_CASES[6], CONV_CASES[7], CONV_CASES[8],
                                  (2, 9, 11, 32, 40, 3, 2, 1, 2), (3, 6, 5, 8, 12, 3, 1, 0, 3)])
def test_conv_fwd_wide_mfma_fp32_vs_fp64(case, v):
    """The 32x32x16-MFMA forward twins (igemm_nt32 / pipe_nt32 WIDE: every
    tile shape, register-staged and ring, with and without split-K, aligned
    and generic gathers), pinned, vs an fp64 conv."""
    from cerebro_ds_kpgi_amd.ops import _hip
    B, H, W, cin, cout, k, s, p, G = case
    spec = ParamSpec("w", (cout, k, k, cin), "weight", fan_in=k * k * cin)
    a, refs = _make([spec], G)
    torch.manual_seed(1)
    x = torch.randn(B, H, W, G * cin, device="cuda")
    _hip.conv_set_variant(0, v)
    try:
        y = P.conv2d(x, refs["w"], s, p)
        torch.cuda.synchronize()
    finally:
        _hip.conv_set_variant(0, -1)
    y64 = F.conv2d(_nchw(x.double()), _w64(refs["w"]), None, s, p, 1, G)
    e = _rel(y, _nhwc(y64))
    print("wide fwd", case, v, "rel err %.2e" % e)
    assert e < TOL, e


@pytest.mark.parametrize("v", [12, 13, 14, 18, 19, 20])
def test_conv_bn_unit_wide_fwd_fp32_vs_fp64(v):
    """BN statistics from the wide forward epilogue (epi32w's 32-lane row
    reduction): the fused unit with the forward pinned to a wide variant."""
    from cerebro_ds_kpgi_amd.ops import _hip
    _hip.conv_set_variant(0, v)
    try:
        test_conv_bn_unit_fp32_vs_fp64(True, True, False)
    finally:
        _hip.conv_set_variant(0, -1)


@pytest.mark.parametrize("vd,vw", [(12, 12), (13, 13), (14, 14), (18, 12), (19, 13), (20, 14)])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_bwd_wide_mfma_fp32_vs_fp64(case, vd, vw):
    """The 32x32x16-MFMA dgrad (igemm_nn32 WIDE, tn_frag32 transposed reads of
    the tn_off_w image) and wgrad (wgrad_reg_body32 WIDE) twins, pinned, on
    every conv case (incl. split-K, strided, generic-gather fallbacks)."""
    from cerebro_ds_kpgi_amd.ops import _hip
    _hip.conv_set_variant(1, vd)
    _hip.conv_set_variant(2, vw)
    try:
        test_conv_fp32_vs_fp64(case)
    finally:
        _hip.conv_set_variant(1, -1)
        _hip.conv_set_variant(2, -1)


@pytest.mark.parametrize("v", [24, 26, 30, 32])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_intra_block_ksplit_fp32_vs_fp64(case, v):
    """The intra-block K-split twins (512-thread igemm_nt32 / igemm_nn32 with
    WG = 2: two wave groups on the halves of the K range, LDS hand-off of the
    accumulators), fwd and dgrad pinned, with and without split-K, on every
    conv case (odd K-tile counts: the last group's surplus step is masked)."""
    from cerebro_ds_kpgi_amd.ops import _hip
    _hip.conv_set_variant(0, v)
    _hip.conv_set_variant(1, v)
    try:
        test_conv_fp32_vs_fp64(case)
    finally:
        _hip.conv_set_variant(0, -1)
        _hip.conv_set_variant(1, -1)


@pytest.mark.parametrize("v", [24, 26, 30])
def test_conv_bn_unit_ksplit_fp32_vs_fp64(v):
    """BN statistics (fwd epilogue) and the BN-link dgrad epilogue from the
    K-split kernels' surviving wave group."""
    from cerebro_ds_kpgi_amd.ops import _hip
    _hip.conv_set_variant(0, v)
    _hip.conv_set_variant(1, v)
    try:
        test_conv_bn_unit_fp32_vs_fp64(True, True, False)
        test_bn_link_dgrad_epilogue_fp32()
    finally:
        _hip.conv_set_variant(0, -1)
        _hip.conv_set_variant(1, -1)


@pytest.mark.parametrize("narrow", [1, 0, 2])
@pytest.mark.parametrize("vb", [1, 12, 13, 14])
def test_wgrad_batch_wide_fp32_vs_fp64(vb, narrow):
    """Batched (deferred) fp32 weight gradients on the register 128x128 and
    the wide kernels (cer_wgrad_batch_flush with ids 1, 12-14) over three
    layers at once; ``narrow``: the 64-output-channel layer goes to its own
    64x128-tile launch (CER_WGB_NARROW=2, the default), to a 64x64-tile one
    (1) or stays in the batch (0)."""
    from cerebro_ds_kpgi_amd.ops import _hip, streams
    # N = 64 (its own 64x64 launch), a K = 64 1x1 layer and two wide layers
    cases = [CONV_CASES[0], CONV_CASES[1], CONV_CASES[5], (8, 14, 14, 64, 256, 1, 1, 0, 4)]
    keep = streams._BATCH_VARIANT
    streams.set_batch_variant(vb)
    _hip.lib().cer_wgrad_batch_set_narrow(narrow)
    try:
        errs = []
        made = []
        for (B, H, W, cin, cout, k, s, p, G) in cases:
            spec = ParamSpec("w", (cout, k, k, cin), "weight", fan_in=k * k * cin)
            a, refs = _make([spec], G)
            torch.manual_seed(1)
            x = torch.randn(B, H, W, G * cin, device="cuda").requires_grad_(True)
            made.append((a, refs, x, (B, H, W, cin, cout, k, s, p, G)))
        with streams.deferred_wgrad():
            for a, refs, x, c in made:
                y = P.conv2d(x, refs["w"], c[6], c[7])
                torch.manual_seed(3)
                y.backward(torch.randn_like(y))
        torch.cuda.synchronize()
        for a, refs, x, (B, H, W, cin, cout, k, s, p, G) in made:
            torch.manual_seed(3)
            w64 = _w64(refs["w"]).requires_grad_(True)
            y64 = F.conv2d(_nchw(x.detach().double()), w64, None, s, p, 1, G)
            y64.backward(_nchw(torch.randn(y64.shape[0], y64.shape[2], y64.shape[3], y64.shape[1],
                                           device="cuda").double()))
            dw64 = w64.grad.view(G, cout, cin, k, k).permute(0, 1, 3, 4, 2)
            errs.append(_rel(a.grad.view(G, -1)[:, :dw64[0].numel()], dw64.reshape(G, -1)))
    finally:
        streams.set_batch_variant(keep)
        _hip.lib().cer_wgrad_batch_set_narrow(2)
    print("wgrad batch wide", vb, narrow, ["%.1e" % e for e in errs])
    assert max(errs) < TOL, errs


@pytest.mark.parametrize("vd", [12, 13, 14])
def test_bn_link_dgrad_epilogue_wide_fp32(vd):
    """BN-backward partials from the wide dgrad epilogue (epi32w BSTAT)."""
    from cerebro_ds_kpgi_amd.ops import _hip
    _hip.conv_set_variant(1, vd)
    try:
        test_bn_link_dgrad_epilogue_fp32()
    finally:
        _hip.conv_set_variant(1, -1)


@pytest.mark.parametrize("act,res,stem", [(True, False, False), (True, True, False),
                                          (False, False, False), (True, False, True)])
def test_conv_bn_unit_fp32_vs_fp64(act, res, stem):
    """The fused training unit act(BN(conv(x)) + residual): conv epilogue BN
    statistics, BN apply, BN backward, dgrad (with BN-link partials when the
    output feeds another unit), wgrad, running statistics."""
    if stem:
        B, H, cin, cout, k, s, p, G = 32, 112, 3, 64, 7, 2, 3, 8
    else:
        B, H, cin, cout, k, s, p, G = 32, 14, 128, 256, 3, 1, 1, 8
    specs = [ParamSpec("w", (cout, k, k, cin), "weight", fan_in=k * k * cin),
             ParamSpec("g", (cout,), "gamma"), ParamSpec("b", (cout,), "beta"),
             ParamSpec("rm", (cout,), "running_mean"), ParamSpec("rv", (cout,), "running_var")]
    a, refs = _make(specs, G, seed=7)
    rm0 = refs["rm"].master().clone()
    rv0 = refs["rv"].master().clone()
    torch.manual_seed(2)
    x = torch.randn(B, H, H, G * cin, device="cuda")
    Ho = (H + 2 * p - k) // s + 1
    r = torch.randn(B, Ho, Ho, G * cout, device="cuda") if res else None
    xx = x.clone().requires_grad_(not stem)
    rr = r.clone().requires_grad_(True) if res else None
    anchor = torch.zeros((), device="cuda", requires_grad=True)
    y = P.conv_bn_act(xx, refs["w"], refs["g"], refs["b"], refs["rm"], refs["rv"], s, p, act,
                      rr, 0.1, 1e-5, anchor=anchor)
    torch.manual_seed(3)
    gy = torch.randn_like(y)
    y.backward(gy)
    torch.cuda.synchronize()
    # fp64 reference
    x64 = _nchw(x.double()).requires_grad_(not stem)
    w64 = _w64(refs["w"]).requires_grad_(True)
    g64 = refs["g"].master().double().reshape(-1).requires_grad_(True)
    b64 = refs["b"].master().double().reshape(-1).requires_grad_(True)
    r64 = _nchw(r.double()).requires_grad_(True) if res else None
    z64 = F.conv2d(x64, w64, None, s, p, 1, G)
    mean = z64.mean((0, 2, 3))
    var = z64.var((0, 2, 3), unbiased=False)
    zh = (z64 - mean.view(1, -1, 1, 1)) / torch.sqrt(var.view(1, -1, 1, 1) + 1e-5)
    o = zh * g64.view(1, -1, 1, 1) + b64.view(1, -1, 1, 1)
    if res:
        o = o + r64
    if act:
        o = o * _nchw((y > 0).double())      # our forward's ReLU mask (module docstring)
    o.backward(_nchw(gy.double()))
    n = z64.numel() // z64.shape[1]
    if act:
        o = torch.relu(o)
    errs = {"y": _rel(y, _nhwc(o.detach())),
            "dW": _rel(refs["w"].grad(), w64.grad.view(G, cout, cin, k, k).permute(0, 1, 3, 4, 2)),
            "dgamma": _rel(refs["g"].grad().reshape(-1), g64.grad),
            "dbeta": _rel(refs["b"].grad().reshape(-1), b64.grad),
            "rmean": _rel(refs["rm"].master().reshape(-1),
                          0.9 * rm0.reshape(-1).double() + 0.1 * mean.detach()),
            "rvar": _rel(refs["rv"].master().reshape(-1),
                         0.9 * rv0.reshape(-1).double() + 0.1 * var.detach() * n / (n - 1))}
    if not stem:
        errs["dx"] = _rel(xx.grad, _nhwc(x64.grad))
    if res:
        errs["dres"] = _rel(rr.grad, _nhwc(r64.grad))
    print("conv_bn", act, res, stem, {k_: "%.1e" % v for k_, v in errs.items()})
    assert max(errs.values()) < TOL, errs


def test_bn_link_dgrad_epilogue_fp32():
    """Two stacked units (a ResNet bottleneck step): the second unit's dgrad
    epilogue computes the first BN's backward partials (BNLink)."""
    B, H, C, G = 32, 14, 64, 8
    specs = []
    for i in (1, 2):
        specs += [ParamSpec("w%d" % i, (C, 3, 3, C), "weight", fan_in=9 * C),
                  ParamSpec("g%d" % i, (C,), "gamma"), ParamSpec("b%d" % i, (C,), "beta"),
                  ParamSpec("rm%d" % i, (C,), "running_mean"),
                  ParamSpec("rv%d" % i, (C,), "running_var")]
    a, R = _make(specs, G, seed=11)
    torch.manual_seed(5)
    x = torch.randn(B, H, H, G * C, device="cuda").requires_grad_(True)
    h = P.conv_bn_act(x, R["w1"], R["g1"], R["b1"], R["rm1"], R["rv1"], 1, 1, True, None,
                      0.1, 1e-5, link_out=True)
    y = P.conv_bn_act(h, R["w2"], R["g2"], R["b2"], R["rm2"], R["rv2"], 1, 1, True, None,
                      0.1, 1e-5)
    gy = torch.randn_like(y)
    y.backward(gy)
    torch.cuda.synchronize()

    def unit(inp, w, g, b, ours):
        z = F.conv2d(inp, w, None, 1, 1, 1, G)
        m = z.mean((0, 2, 3)).view(1, -1, 1, 1)
        v = z.var((0, 2, 3), unbiased=False).view(1, -1, 1, 1)
        o = (z - m) / torch.sqrt(v + 1e-5) * g.view(1, -1, 1, 1) + b.view(1, -1, 1, 1)
        return o * _nchw((ours > 0).double())    # our forward's ReLU mask
    x64 = _nchw(x.detach().double()).requires_grad_(True)
    P64 = {}
    for i in (1, 2):
        P64["w%d" % i] = _w64(R["w%d" % i]).requires_grad_(True)
        P64["g%d" % i] = R["g%d" % i].master().double().reshape(-1).requires_grad_(True)
        P64["b%d" % i] = R["b%d" % i].master().double().reshape(-1).requires_grad_(True)
    o = unit(unit(x64, P64["w1"], P64["g1"], P64["b1"], h.detach()), P64["w2"], P64["g2"],
             P64["b2"], y.detach())
    o.backward(_nchw(gy.double()))
    errs = {"y": _rel(y, _nhwc(torch.relu(o.detach()))), "dx": _rel(x.grad, _nhwc(x64.grad)),
            "dgamma1": _rel(R["g1"].grad().reshape(-1), P64["g1"].grad),
            "dbeta1": _rel(R["b1"].grad().reshape(-1), P64["b1"].grad),
            "dW1": _rel(R["w1"].grad(),
                        P64["w1"].grad.view(G, C, C, 3, 3).permute(0, 1, 3, 4, 2))}
    print("bn_link", {k_: "%.1e" % v for k_, v in errs.items()})
    assert max(errs.values()) < TOL, errs


def test_bn_link_strided_gradjoin_inplace_fp32(monkeypatch):
    """A ResNet stage transition: a BN output h feeds two strided 1x1 convs
    (c1 and the projection shortcut) joined by a GradJoin.  The second dgrad
    accumulates into the first one's dx IN PLACE (consume_addend) and is
    BN-linked (it carries h's whole gradient).  The first dx is zero off the
    stride grid, so the second dgrad's epilogue computes h's BN partials
    (conv.hip g_addend_grid) and h's BN skips its own pass.  dx, dgamma /
    dbeta of h's BN and both weight gradients against fp64 autograd."""
    from cerebro_ds_kpgi_amd.ops import _hip
    used = []
    real = _hip.bn_act_bwd

    def spy(*a, **k):
        used.append(k.get("part") is not None)
        return real(*a, **k)
    monkeypatch.setattr(_hip, "bn_act_bwd", spy)
    B, H, C, G = 8, 14, 64, 2
    Co1, Co2 = 32, 128
    specs = [ParamSpec("w0", (C, 3, 3, C), "weight", fan_in=9 * C),
             ParamSpec("g0", (C,), "gamma"), ParamSpec("b0", (C,), "beta"),
             ParamSpec("rm0", (C,), "running_mean"), ParamSpec("rv0", (C,), "running_var")]
    for i, co in ((1, Co1), (2, Co2)):
        specs += [ParamSpec("w%d" % i, (co, 1, 1, C), "weight", fan_in=C),
                  ParamSpec("g%d" % i, (co,), "gamma"), ParamSpec("b%d" % i, (co,), "beta"),
                  ParamSpec("rm%d" % i, (co,), "running_mean"),
                  ParamSpec("rv%d" % i, (co,), "running_var")]
    a, R = _make(specs, G, seed=13)
    torch.manual_seed(9)
    x = torch.randn(B, H, H, G * C, device="cuda").requires_grad_(True)
    h = P.conv_bn_act(x, R["w0"], R["g0"], R["b0"], R["rm0"], R["rv0"], 1, 1, True, None,
                      0.1, 1e-5, link_out=True)
    j = P.GradJoin()
    y1 = P.conv_bn_act(h, R["w1"], R["g1"], R["b1"], R["rm1"], R["rv1"], 2, 0, True, None,
                       0.1, 1e-5, join=j)
    y2 = P.conv_bn_act(h, R["w2"], R["g2"], R["b2"], R["rm2"], R["rv2"], 2, 0, False, None,
                       0.1, 1e-5, join=j)
    g1, g2 = torch.randn_like(y1), torch.randn_like(y2)
    (y1 * g1).sum().add_((y2 * g2).sum()).backward()
    torch.cuda.synchronize()
    # h's BN (the first unit) runs its backward last: with the epilogue's partials
    assert used and used[-1], used

    def unit(inp, w, g, b, st, pad, mask):
        z = F.conv2d(inp, w, None, st, pad, 1, G)
        m = z.mean((0, 2, 3)).view(1, -1, 1, 1)
        v = z.var((0, 2, 3), unbiased=False).view(1, -1, 1, 1)
        o = (z - m) / torch.sqrt(v + 1e-5) * g.view(1, -1, 1, 1) + b.view(1, -1, 1, 1)
        return o if mask is None else o * _nchw((mask > 0).double())
    x64 = _nchw(x.detach().double()).requires_grad_(True)
    P64 = {}
    for i in (0, 1, 2):
        P64["w%d" % i] = _w64(R["w%d" % i]).requires_grad_(True)
        P64["g%d" % i] = R["g%d" % i].master().double().reshape(-1).requires_grad_(True)
        P64["b%d" % i] = R["b%d" % i].master().double().reshape(-1).requires_grad_(True)
    h64 = unit(x64, P64["w0"], P64["g0"], P64["b0"], 1, 1, h.detach())
    o1 = unit(h64, P64["w1"], P64["g1"], P64["b1"], 2, 0, y1.detach())
    o2 = unit(h64, P64["w2"], P64["g2"], P64["b2"], 2, 0, None)
    ((o1 * _nchw(g1.double())).sum() + (o2 * _nchw(g2.double())).sum()).backward()
    errs = {"dx": _rel(x.grad, _nhwc(x64.grad)),
            "dgamma0": _rel(R["g0"].grad().reshape(-1), P64["g0"].grad),
            "dbeta0": _rel(R["b0"].grad().reshape(-1), P64["b0"].grad),
            "dW0": _rel(R["w0"].grad(), P64["w0"].grad.view(G, C, C, 3, 3).permute(0, 1, 3, 4, 2)),
            "dW1": _rel(R["w1"].grad(), P64["w1"].grad.view(G, Co1, C, 1, 1).permute(0, 1, 3, 4, 2)),
            "dW2": _rel(R["w2"].grad(), P64["w2"].grad.view(G, Co2, C, 1, 1).permute(0, 1, 3, 4, 2))}
    print("bn_link strided gradjoin", {k_: "%.1e" % v for k_, v in errs.items()})
    assert max(errs.values()) < TOL, errs


@pytest.mark.parametrize("B,K,N,G,relu", [(32, 2048, 1000, 8, False), (256, 1000, 500, 4, True),
                                          (64, 500, 2, 3, False), (32, 4096, 4096, 2, True)])
def test_linear_fp32_vs_fp64(B, K, N, G, relu):
    specs = [ParamSpec("w", (N, K), "weight", fan_in=K), ParamSpec("b", (N,), "bias")]
    a, R = _make(specs, G, seed=3)
    torch.manual_seed(4)
    x = torch.randn(B, G * K, device="cuda").requires_grad_(True)
    y = P.linear(x, R["w"], R["b"], relu)
    gy = torch.randn_like(y)
    y.backward(gy)
    torch.cuda.synchronize()
    x64 = x.detach().double().view(B, G, K).transpose(0, 1).requires_grad_(True)
    w64 = R["w"].master().double().requires_grad_(True)
    b64 = R["b"].master().double().requires_grad_(True)
    z = torch.bmm(x64, w64.transpose(1, 2)) + b64.unsqueeze(1)
    if relu:
        z = torch.relu(z)
    z.backward(gy.double().view(B, G, N).transpose(0, 1))
    errs = {"y": _rel(y, z.detach().transpose(0, 1).reshape(B, G * N)),
            "dx": _rel(x.grad, x64.grad.transpose(0, 1).reshape(B, G * K)),
            "dW": _rel(R["w"].grad(), w64.grad), "db": _rel(R["b"].grad(), b64.grad)}
    print("linear", B, K, N, G, {k_: "%.1e" % v for k_, v in errs.items()})
    assert max(errs.values()) < TOL, errs


def test_pools_fp32_vs_fp64():
    torch.manual_seed(6)
    x = torch.randn(32, 56, 56, 8 * 64, device="cuda").requires_grad_(True)
    y = P.maxpool2d(x, 3, 2, 1)
    gy = torch.randn_like(y)
    y.backward(gy)
    x64 = _nchw(x.detach().double()).requires_grad_(True)
    y64 = F.max_pool2d(x64, 3, 2, 1)
    y64.backward(_nchw(gy.double()))
    assert _rel(y, _nhwc(y64.detach())) < 1e-7
    assert _rel(x.grad, _nhwc(x64.grad)) < 1e-7
    x2 = torch.randn(32, 4, 4, 8 * 2048, device="cuda").requires_grad_(True)
    g = P.global_avgpool(x2)
    gg = torch.randn_like(g)
    g.backward(gg)
    x64 = x2.detach().double().requires_grad_(True)
    g64 = x64.mean((1, 2))
    g64.backward(gg.double())
    assert _rel(g, g64.detach()) < 1e-6
    assert _rel(x2.grad, x64.grad) < 1e-6
    x3 = torch.randn(8, 14, 14, 3 * 32, device="cuda").requires_grad_(True)
    a3 = P.avgpool2d(x3, 3, 1, 1, count_include_pad=False)
    ga = torch.randn_like(a3)
    a3.backward(ga)
    # contiguous NCHW: PyTorch-ROCm's avg_pool2d backward on a channels-last
    # view with padding is wrong (ops/nn.py avgpool2d)
    x64 = _nchw(x3.detach().double()).contiguous().requires_grad_(True)
    a64 = F.avg_pool2d(x64, 3, 1, 1, count_include_pad=False)
    a64.backward(_nchw(ga.double()))
    assert _rel(a3, _nhwc(a64.detach())) < 1e-6
    assert _rel(x3.grad, _nhwc(x64.grad)) < 1e-6


def test_dwconv_fp32_vs_fp64():
    G, C, B, H = 2, 96, 8, 28
    spec = ParamSpec("w", (C, 3, 3), "weight", fan_in=9)
    a, R = _make([spec], G, seed=9)
    torch.manual_seed(8)
    x = torch.randn(B, H, H, G * C, device="cuda").requires_grad_(True)
    y = P.dwconv2d(x, R["w"], 2, (0, 1, 0, 1))
    gy = torch.randn_like(y)
    y.backward(gy)
    x64 = _nchw(x.detach().double()).requires_grad_(True)
    w64 = R["w"].master().double().reshape(G * C, 1, 3, 3).requires_grad_(True)
    y64 = F.conv2d(F.pad(x64, (0, 1, 0, 1)), w64, None, 2, 0, 1, G * C)
    y64.backward(_nchw(gy.double()))
    errs = (_rel(y, _nhwc(y64.detach())), _rel(x.grad, _nhwc(x64.grad)),
            _rel(R["w"].grad().reshape(G * C, 1, 3, 3), w64.grad))
    assert max(errs) < 1e-5, errs


def test_embedding_bag_fp32_vs_fp64():
    G, B, nnz, K, N = 4, 64, 39, 7306, 1000
    specs = [ParamSpec("w", (K, N), "weight", fan_in=K), ParamSpec("b", (N,), "bias")]
    a, R = _make(specs, G, seed=12)
    torch.manual_seed(9)
    idx = torch.randint(0, K, (G, B, nnz), device="cuda", dtype=torch.int32)
    idx[:, :, -3:] = -1
    y = P.embedding_bag(idx, R["w"], R["b"], True,
                        anchor=torch.zeros((), device="cuda", requires_grad=True))
    assert y.dtype == torch.float32
    gy = torch.randn_like(y)
    y.backward(gy)
    torch.cuda.synchronize()
    w64 = R["w"].master().double().requires_grad_(True)
    b64 = R["b"].master().double().requires_grad_(True)
    rows = torch.stack([w64[g][idx[g].long().clamp(min=0)] for g in range(G)])
    z = (rows * (idx >= 0).unsqueeze(-1).double()).sum(2) + b64.unsqueeze(1)
    z = z * (y.detach().view(B, G, N).transpose(0, 1) > 0).double()   # our ReLU mask
    z.backward(gy.double().view(B, G, N).transpose(0, 1))
    errs = (_rel(y, z.detach().transpose(0, 1).reshape(B, G * N)),
            _rel(R["w"].grad(), w64.grad), _rel(R["b"].grad(), b64.grad))
    assert max(errs) < 1e-5, errs


def test_gather_fp32_exact():
    from cerebro_ds_kpgi_amd.data.store import PartitionStore, gather_batch, input_buffers
    st = PartitionStore("imagenet", [0, 1], 128, 32, "cuda")
    st.new_epoch(1)
    part = torch.tensor([1, 0, 1], dtype=torch.int32, device="cuda")
    cur = torch.tensor([2], dtype=torch.int32, device="cuda")
    x1, y1 = input_buffers(st, 3, 16, torch.float32)
    x2, y2 = input_buffers(st, 3, 16, torch.float32)
    gather_batch(st, True, part, cur, 16, x1, y1)
    backend.force_torch_ops(["gather"])
    gather_batch(st, True, part, cur, 16, x2, y2)
    backend.force_torch_ops([])
    assert torch.equal(y1, y2)
    torch.testing.assert_close(x1, x2, rtol=1e-6, atol=1e-6)


def test_resnet50_trajectory_fp32_hip_vs_oracle():
    """200 Adam steps of ResNet-50 (2 packed configs) on a fixed stream of
    batches: the fp32 HIP path (HIP graph replayed) and the fp32 PyTorch /
    MIOpen oracle path follow the same loss trajectory."""
    from cerebro_ds_kpgi_amd.models import create_model_from_mst
    from cerebro_ds_kpgi_amd.ops.loss import softmax_ce
    from cerebro_ds_kpgi_amd.ops.optim import optimizer_step
    G, B, steps = 2, 16, 200
    torch.manual_seed(21)
    nbatch = 64
    xs = torch.randn(nbatch, B, 112, 112, 3 * G, device="cuda")
    ys = torch.randint(0, 10, (nbatch, G, B), device="cuda", dtype=torch.int32)
    curves = []
    for force in ([], ["conv", "bn", "pool", "bias", "linear", "loss", "adam"]):
        backend.force_torch_ops(force)
        net = create_model_from_mst({"model": "resnet50"})
        a = Arena(net.layout, G, "cuda", torch.float32)
        for g in range(G):
            a.init_model(g, 2018 + g)
            a.set_hparams(g, 1e-4, 1e-4)
        net.bind(a)
        acc = torch.zeros(G, 4, device="cuda")
        losses = []
        for it in range(steps):
            loss = softmax_ce(net.forward(xs[it % nbatch], True), ys[it % nbatch], acc, G)
            loss.sum().backward()
            optimizer_step(a, "adam", l2=True)
            losses.append(loss.detach())
        curves.append(torch.stack(losses).cpu())
        backend.force_torch_ops([])
    hip, ref = curves
    assert torch.isfinite(hip).all()
    # the model memorises the batches: both curves fall well below ln(10)
    assert hip[-20:].mean() < 0.5 * hip[:20].mean()
    # 20-step window means, deviation relative to the initial loss level
    wh, wr = hip.view(10, 20, G).mean(1), ref.view(10, 20, G).mean(1)
    dev = ((wh - wr).abs() / ref[:20].mean(0)).max().item()
    print("trajectory window means hip", wh[:, 0].tolist(), "ref", wr[:, 0].tolist(),
          "max dev %.2e" % dev)
    assert dev < 2e-2, dev


@pytest.mark.parametrize("B,H,cin,cout,groups,k,s,G", [(4, 14, 128, 128, 32, 3, 1, 2),
                                                     (2, 28, 256, 256, 32, 3, 2, 2),
                                                     (3, 7, 64, 96, 8, 3, 1, 3),
                                                     (2, 9, 48, 48, 4, 1, 1, 2)])
def test_grouped_conv_fp32_vs_fp64(B, H, cin, cout, groups, k, s, G):
    """ResNeXt grouped conv on the HIP kernels (per-config launches over the
    groups, conv.hip cer_conv_grouped_*): y, dx, dW vs fp64 torch grouped conv,
    inside and outside the deferred weight-gradient batch."""
    from cerebro_ds_kpgi_amd.ops import _hip, streams
    from cerebro_ds_kpgi_amd.ops.backend import take_fallbacks
    p = k // 2
    spec = ParamSpec("w", (cout, k, k, cin // groups), "weight", fan_in=k * k * cin // groups)
    for batched in (False, True):
        a, R = _make([spec], G, seed=21)
        a.grad_clean = True
        torch.manual_seed(2)
        x = torch.randn(B, H, H, G * cin, device="cuda").requires_grad_(True)
        take_fallbacks()
        with streams.deferred_wgrad(batched):
            y = P.grouped_conv2d(x, R["w"], s, p, groups)
            gy = torch.randn_like(y)
            y.backward(gy)
        streams.join()
        torch.cuda.synchronize()
        assert not take_fallbacks(), "grouped conv fell back to PyTorch"
        w64 = _w64(R["w"]).requires_grad_(True)
        x64 = _nchw(x.detach().double()).requires_grad_(True)
        y64 = F.conv2d(x64, w64, None, s, p, 1, G * groups)
        y64.backward(_nchw(gy.double()))
        errs = {"y": _rel(y, _nhwc(y64.detach())), "dx": _rel(x.grad, _nhwc(x64.grad)),
                "dW": _rel(R["w"].grad(), w64.grad.view(G, cout, cin // groups, k, k)
                           .permute(0, 1, 3, 4, 2))}
        print("grouped", (B, H, cin, cout, groups, k, s, G, batched),
              {kk: "%.1e" % v for kk, v in errs.items()})
        assert max(errs.values()) < TOL, errs


def test_resnext101_trains_on_hip_under_graph():
    """Every op of resnext101 (grouped 3x3 convs included) runs on our HIP
    kernels, so its step is captured as a HIP graph (round-2 VERDICT item 9)."""
    from cerebro_ds_kpgi_amd.ops.backend import take_fallbacks
    from cerebro_ds_kpgi_amd.parallel import init_distributed
    from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine
    bs = 4
    msts = [{"learning_rate": lr, "lambda_value": 1e-4, "batch_size": bs, "model": "resnext101"}
            for lr in (1e-4, 1e-5)]
    take_fallbacks()
    eng = MOPEngine(msts, init_distributed(), EngineOptions(
        n_train=16 * bs, n_valid=2 * bs, slots_per_gpu=2, verbose=False, ckpt_every="none",
        compute_dtype="fp32", shuffle=False))
    eng.sched.start_epoch(1)
    eng.store.new_epoch(1)
    eng._hop_and_load(eng.sched.next_round())
    w = list(eng.groups.values())[0].current
    w.prepare(True)
    w.train_steps(6)
    torch.cuda.synchronize()
    assert not w.eager_only, "resnext101 fell back to eager (PyTorch ops)"
    assert w.graph is not None, "the step was not captured"
    assert torch.isfinite(w.arena.state).all()
    eng.close()


@pytest.mark.parametrize("act,res", [(True, False), (False, False), (True, True)])
@pytest.mark.parametrize("shape,G", [((8, 56, 56, 64), 1), ((16, 28, 28, 2 * 256), 2)])
def test_bn_bwd_fp64_slabs_match_staged_fp32(act, res, shape, G, monkeypatch):
    """BN backward of a layer with many row slabs (no dgrad-epilogue link):
    partials by fp64 atomics into STAT_SLABS slabs, finalize folded into the
    apply (bn.hip cer_bn_set_bwd_f64) == fp32 per-slab partials + separate
    finalize, and both == an fp64 reference."""
    from cerebro_ds_kpgi_amd.ops import _hip
    C = shape[-1] // G
    M = shape[0] * shape[1] * shape[2]
    assert _hip.lib().cer_bn_bwd_f64_floats(M, shape[-1], C, _hip.STAT_SLABS) > 0
    specs = [ParamSpec("g", (C,), "gamma"), ParamSpec("b", (C,), "beta"),
             ParamSpec("rm", (C,), "running_mean"), ParamSpec("rv", (C,), "running_var")]
    torch.manual_seed(17)
    x = 2 * torch.randn(shape, device="cuda") + 0.3
    r = torch.randn(shape, device="cuda") if res else None
    gy = torch.randn(shape, device="cuda")
    outs = []
    for slabs in (_hip.STAT_SLABS, 0):
        monkeypatch.setattr(_hip, "STAT_SLABS", slabs)
        a, refs = _make(specs, G, seed=5)
        a.grad_clean = True
        a.grad.zero_()
        xx = x.clone().requires_grad_(True)
        rr = r.clone().requires_grad_(True) if res else None
        y = P.bn_act(xx, refs["g"], refs["b"], refs["rm"], refs["rv"], True, act, rr)
        y.backward(gy)
        torch.cuda.synchronize()
        outs.append((y.detach(), xx.grad, rr.grad if res else None, a.grad.clone()))
    # fp64 reference of the same op (training BN, act under OUR forward mask)
    gam = refs["g"].master().double().reshape(-1)
    bet = refs["b"].master().double().reshape(-1)
    xd = x.double().reshape(-1, shape[-1]).requires_grad_(True)
    mu = xd.mean(0)
    var = xd.var(0, unbiased=False)
    z = (xd - mu) / torch.sqrt(var + 1e-5) * gam + bet
    if res:
        z = z + r.double().reshape(-1, shape[-1])
    mask = (outs[0][0].reshape(-1, shape[-1]) > 0).double() if act else 1.0
    (z * mask * gy.double().reshape(-1, shape[-1])).sum().backward()
    for u, v in zip(outs[0], outs[1]):
        if u is not None:
            assert _rel(u, v) < 1e-5, _rel(u, v)
    e = _rel(outs[0][1].reshape(-1, shape[-1]), xd.grad)
    print("fp64-slab BN backward dx rel vs fp64", e)
    assert e < TOL
