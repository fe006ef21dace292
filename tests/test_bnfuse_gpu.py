"""Conv + BatchNorm forward fused behind a grid barrier (GPU box).

``conv.hip`` BNFwdFuse: when every block of a conv launch is resident at
once (one config per GPU, the N = 8 shape), the conv epilogue adds its BN
statistics into the fp64 slabs, all blocks meet at a grid barrier, and each
block finalizes its channels and applies BN (+ residual, ReLU, HL output,
activation bits) to the tile still in its registers -- no BN kernel.

Checks: the fused unit against an fp64 reference (same bound as
tests/test_fp32_gpu.py), against the unfused path (conv + folded BN apply)
to fp32 rounding, the activation bits and HL output bit-for-bit, that the
fused path actually ran (``FUSE_COUNTS``), that no barrier timed out, and a
one-config ResNet-50 engine run fused vs unfused.
"""

import pytest
import torch
import torch.nn.functional as F

from cerebro_ds_kpgi_amd.ops import backend
from cerebro_ds_kpgi_amd.ops import nn as P
from cerebro_ds_kpgi_amd.runtime.arena import ParamSpec

from test_fp32_gpu import TOL, _make, _nchw, _nhwc, _rel, _w64

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _hip_backend():
    from cerebro_ds_kpgi_amd.ops import _hip
    backend.set_backend("hip")
    backend.force_torch_ops([])
    backend.take_fallbacks()
    yield
    assert not backend.take_fallbacks(), "an op fell back to the PyTorch path"
    _hip.set_bn_fuse(True)
    _hip.stats_step(None)


def _unit(case, fuse, hl=False):
    """One training unit y = act(BN(conv(x)) + res) inside a step's stats
    arena; returns the outputs and gradients."""
    from cerebro_ds_kpgi_amd.ops import _hip
    B, H, cin, cout, k, s, p, G, act, res = case
    specs = [ParamSpec("w", (cout, k, k, cin), "weight", fan_in=k * k * cin),
             ParamSpec("g", (cout,), "gamma"), ParamSpec("b", (cout,), "beta"),
             ParamSpec("rm", (cout,), "running_mean"), ParamSpec("rv", (cout,), "running_var")]
    a, refs = _make(specs, G, seed=11)
    torch.manual_seed(5)
    x = torch.randn(B, H, H, G * cin, device="cuda")
    Ho = (H + 2 * p - k) // s + 1
    r = torch.randn(B, Ho, Ho, G * cout, device="cuda") if res else None
    _hip.set_bn_fuse(fuse)
    arena = _hip.new_stats_arena("cuda")
    out = {}
    for rep in range(2):                 # the second pass reuses the barrier slot
        _hip.stats_step(arena)
        before = dict(_hip.FUSE_COUNTS)
        xx = x.clone().requires_grad_(True)
        rr = r.clone().requires_grad_(True) if res else None
        anchor = torch.zeros((), device="cuda", requires_grad=True)
        y = P.conv_bn_act(xx, refs["w"], refs["g"], refs["b"], refs["rm"], refs["rv"], s, p, act,
                          rr, 0.1, 1e-5, anchor=anchor, hl_out=hl)
        yv = _hip.hl_to_fp32(y) if _hip.is_hl(y) else y
        torch.manual_seed(6)
        gy = torch.randn_like(yv)
        y.backward(gy)
        torch.cuda.synchronize()
        _hip.stats_step(None)
        fused = _hip.FUSE_COUNTS["fused"] - before["fused"]
        out = {"y": yv.detach().clone(), "fused": fused, "hl": _hip.is_hl(y),
               "mask": getattr(y, "_cer_mask", None), "gy": gy,
               "rm": refs["rm"].master().clone(), "rv": refs["rv"].master().clone()}
        out.update(dx=xx.grad.clone(), dw=refs["w"].grad().clone(),
                   dg=refs["g"].grad().clone(), db=refs["b"].grad().clone(),
                   dres=rr.grad.clone() if res else None)
    out["x"], out["r"], out["refs"] = x, r, refs
    assert _hip.bn_fuse_errors() == 0
    return out


# (B, H, cin, cout, k, s, p, G, act, residual): ResNet-50 stage-3 / 4 / 5
# shapes at one config per GPU (the N = 8 per-GPU work)
CASES = [(32, 14, 128, 128, 3, 1, 1, 1, True, False),
         (32, 7, 256, 1024, 1, 1, 0, 1, True, True),
         (32, 14, 512, 256, 1, 2, 0, 1, True, False),
         (32, 4, 512, 2048, 1, 1, 0, 1, False, False),
         (32, 28, 128, 512, 1, 1, 0, 1, True, True)]
FITS = [True, True, True, True, False]      # the last grid exceeds one wave: fallback path


@pytest.mark.parametrize("case,fits", list(zip(CASES, FITS)))
def test_fused_conv_bn_vs_fp64_and_unfused(case, fits):
    B, H, cin, cout, k, s, p, G, act, res = case
    fz = _unit(case, True)
    un = _unit(case, False)
    # a grid that does not fit the GPU at once takes the conv + folded BN
    # apply inside the same entry point
    from cerebro_ds_kpgi_amd.ops import _hip
    assert fz["fused"] == (1 if fits else 0), (fz["fused"], _hip.FUSE_WHY)
    assert un["fused"] == 0
    # fused vs unfused: the same statistics (same fp64 slabs, same rounding)
    cmp = {k_: _rel(fz[k_], un[k_]) for k_ in ("y", "rm", "rv", "dx", "dw", "dg", "db")}
    if res:
        cmp["dres"] = _rel(fz["dres"], un["dres"])
        assert torch.equal(fz["mask"], un["mask"]), "activation bits differ"
    print("fused vs unfused", case, {k_: "%.1e" % v for k_, v in cmp.items()})
    assert max(cmp.values()) < 1e-6, cmp
    # fp64 reference (tests/test_fp32_gpu.py::test_conv_bn_unit_fp32_vs_fp64)
    refs = fz["refs"]
    x64 = _nchw(fz["x"].double())
    z64 = F.conv2d(x64, _w64(refs["w"]), None, s, p, 1, G)
    mean = z64.mean((0, 2, 3))
    var = z64.var((0, 2, 3), unbiased=False)
    zh = (z64 - mean.view(1, -1, 1, 1)) / torch.sqrt(var.view(1, -1, 1, 1) + 1e-5)
    o = zh * refs["g"].master().double().view(1, -1, 1, 1) + \
        refs["b"].master().double().view(1, -1, 1, 1)
    if res:
        o = o + _nchw(fz["r"].double())
    if act:
        o = torch.relu(o)
    err = _rel(fz["y"], _nhwc(o))
    print("fused y vs fp64", case, "%.1e" % err)
    assert err < TOL


@pytest.mark.parametrize("case", [CASES[0], CASES[2]])
def test_fused_conv_bn_hl_output_bitwise(case):
    """HL output (the value's only consumer is a conv): the fused epilogue
    writes the same (hi, lo) bf16 pairs as the folded BN apply."""
    fz = _unit(case, True, hl=True)
    un = _unit(case, False, hl=True)
    assert fz["hl"] and un["hl"] and fz["fused"] == 1
    assert _rel(fz["y"], un["y"]) < 1e-6


def _engine_run(fuse, steps=3):
    from cerebro_ds_kpgi_amd.ops import _hip
    from cerebro_ds_kpgi_amd.parallel import init_distributed
    from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine
    msts = [{"learning_rate": 1e-4, "lambda_value": 1e-4, "batch_size": 32, "model": "resnet50"}]
    before = dict(_hip.FUSE_COUNTS)
    eng = MOPEngine(msts, init_distributed(), EngineOptions(
        n_train=32 * steps, n_valid=32, slots_per_gpu=1, verbose=False, ckpt_every="none",
        shuffle=False, scheduler="rotation", runtime="async", seed=7))
    _hip.set_bn_fuse(fuse)
    eng.run_steps(steps, steps)
    torch.cuda.synchronize()
    grp = next(iter(eng.groups.values()))
    nm = grp.layout.n_master
    state = grp.home.state[:, :nm].clone()          # weights + BN statistics
    counts = {k: _hip.FUSE_COUNTS[k] - before[k] for k in before}
    eng.close()
    return state, counts


def test_fused_resnet50_one_config_matches_unfused():
    """One ResNet-50 config (the N = 8 per-GPU work), eager + captured +
    replayed steps: the fused run takes the fused path for most BN layers and
    ends where the unfused run ends, within the run-to-run noise of the
    unfused path itself (ResNet-50 at init amplifies last-bit differences of
    the fp64-slab statistics, scripts/debug/slab_determinism.py)."""
    from cerebro_ds_kpgi_amd.ops import _hip
    s_u1, c_u = _engine_run(False)
    s_u2, _ = _engine_run(False)
    s_f, c_f = _engine_run(True)
    print("fuse counts fused / unfused run", c_f, c_u, "why", _hip.FUSE_WHY)
    assert c_f["fused"] >= 40 and c_u["fused"] == 0
    assert torch.isfinite(s_f).all()
    floor = _rel(s_u2, s_u1)
    d = _rel(s_f, s_u1)
    print("weights rel diff: fused vs unfused %.2e, unfused vs unfused %.2e" % (d, floor))
    assert d <= max(10 * floor, 1e-5), (d, floor)
    assert _hip.bn_fuse_errors() == 0


# ---------------------------------------------------------------------------
# backward: the BN-link dgrad finishes the linked BN's backward
def _chain(fuse, res, hl, C=128, H=14, G=1):
    """unit1 (-> BN-linked output h, optionally a residual join) -> unit2;
    one training step in a stats arena.  Returns the gradients."""
    from cerebro_ds_kpgi_amd.ops import _hip
    B = 32
    specs = []
    for i in (1, 2):
        specs += [ParamSpec("w%d" % i, (C, 3, 3, C), "weight", fan_in=9 * C),
                  ParamSpec("g%d" % i, (C,), "gamma"), ParamSpec("b%d" % i, (C,), "beta"),
                  ParamSpec("rm%d" % i, (C,), "running_mean"),
                  ParamSpec("rv%d" % i, (C,), "running_var")]
    a, R = _make(specs, G, seed=13)
    torch.manual_seed(8)
    x0 = torch.randn(B, H, H, G * C, device="cuda")
    r0 = torch.randn(B, H, H, G * C, device="cuda") if res else None
    _hip.set_bn_fuse(fuse)
    arena = _hip.new_stats_arena("cuda")
    for rep in range(2):
        _hip.stats_step(arena)
        before = dict(_hip.FUSE_COUNTS)
        x = x0.clone().requires_grad_(True)
        r = r0.clone().requires_grad_(True) if res else None
        h = P.conv_bn_act(x, R["w1"], R["g1"], R["b1"], R["rm1"], R["rv1"], 1, 1, True, r,
                          0.1, 1e-5, link_out=True, hl_out=hl and not res)
        y = P.conv_bn_act(h, R["w2"], R["g2"], R["b2"], R["rm2"], R["rv2"], 1, 1, True, None,
                          0.1, 1e-5)
        torch.manual_seed(9)
        gy = torch.randn_like(y)
        y.backward(gy)
        torch.cuda.synchronize()
        _hip.stats_step(None)
        got = {"dx": x.grad.clone(), "dg1": R["g1"].grad().clone(), "db1": R["b1"].grad().clone(),
               "dw1": R["w1"].grad().clone(), "dw2": R["w2"].grad().clone(),
               "bwd_fused": _hip.FUSE_COUNTS["bwd_fused"] - before["bwd_fused"],
               "bwd_unfused": _hip.FUSE_COUNTS["bwd_unfused"] - before["bwd_unfused"]}
        if res:
            got["dres"] = r.grad.clone()
    got.update(x0=x0, r0=r0, R=R, gy=gy, h=h.detach(), y=y.detach())
    assert _hip.bn_fuse_errors() == 0
    return got


@pytest.mark.parametrize("res,hl", [(False, False), (False, True), (True, False)])
def test_fused_bn_backward_vs_unfused_and_fp64(res, hl):
    fz = _chain(True, res, hl)
    un = _chain(False, res, hl)
    assert fz["bwd_fused"] == 1 and un["bwd_fused"] == 0 and un["bwd_unfused"] == 0
    keys = ["dx", "dg1", "db1", "dw1", "dw2"] + (["dres"] if res else [])
    cmp = {k: _rel(fz[k], un[k]) for k in keys}
    print("bwd fused vs unfused", res, hl, {k: "%.1e" % v for k, v in cmp.items()})
    assert max(cmp.values()) < 1e-5, cmp
    # fp64 reference of the chain
    R, G = fz["R"], 1
    from cerebro_ds_kpgi_amd.ops import _hip
    hv = _hip.hl_to_fp32(fz["h"]) if _hip.is_hl(fz["h"]) else fz["h"]

    def unit(inp, w, g, b, ours, resid=None):
        z = F.conv2d(inp, w, None, 1, 1, 1, G)
        m = z.mean((0, 2, 3)).view(1, -1, 1, 1)
        v = z.var((0, 2, 3), unbiased=False).view(1, -1, 1, 1)
        o = (z - m) / torch.sqrt(v + 1e-5) * g.view(1, -1, 1, 1) + b.view(1, -1, 1, 1)
        if resid is not None:
            o = o + resid
        return o * _nchw((ours > 0).double())
    x64 = _nchw(fz["x0"].double()).requires_grad_(True)
    r64 = _nchw(fz["r0"].double()).requires_grad_(True) if res else None
    P64 = {}
    for i in (1, 2):
        P64["w%d" % i] = _w64(R["w%d" % i]).requires_grad_(True)
        P64["g%d" % i] = R["g%d" % i].master().double().reshape(-1).requires_grad_(True)
        P64["b%d" % i] = R["b%d" % i].master().double().reshape(-1).requires_grad_(True)
    o = unit(unit(x64, P64["w1"], P64["g1"], P64["b1"], hv, r64), P64["w2"], P64["g2"],
             P64["b2"], fz["y"])
    o.backward(_nchw(fz["gy"].double()))
    errs = {"dx": _rel(fz["dx"], _nhwc(x64.grad)),
            "dgamma1": _rel(fz["dg1"].reshape(-1), P64["g1"].grad),
            "dbeta1": _rel(fz["db1"].reshape(-1), P64["b1"].grad)}
    if res:
        errs["dres"] = _rel(fz["dres"], _nhwc(r64.grad))
    print("bwd fused vs fp64", {k: "%.1e" % v for k, v in errs.items()})
    assert max(errs.values()) < TOL, errs
