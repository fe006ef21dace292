"""Roofline of a training step: analytic work per kernel family vs measured time.

    python -m cerebro_ds_kpgi_amd.tools.roofline gpurun_out/prof --model resnet50 \
        --configs 8 --batch 32 --dtype fp32 --last-steps 10

Work is traced on the CPU (one eager forward of the architecture at batch 1
through the PyTorch path, every GEMM-shaped op recorded with its shapes) and
scaled to ``configs x batch``:

* conv / linear FLOPs: fwd = 2*M*N*K per layer; dgrad the same (not for the
  first layer, whose input needs no gradient); wgrad the same;
* BatchNorm bytes: per BN element, fwd reads z and writes y, bwd reads dy and
  z and writes dz (statistics come out of the conv epilogue) = 5 x elem size;
* optimizer bytes: Adam reads params, grad, m, v and writes params, m, v and
  the cleared gradient = 32 B per trainable parameter (fp32 arena).

Peaks (MI355X, /opt/skills/guides/MI355X_MICROARCH.md): 2.5 PF dense bf16
MFMA; fp32 mode runs every GEMM as 3 bf16 MFMA passes (hi*hi + hi*lo +
lo*hi), so its MFMA-issued FLOPs are 3x the fp32 FLOPs (ceiling 833 TF
fp32-equivalent; the f32 MFMA peak would be 157 TF); HBM 8 TB/s spec,
~6.3 TB/s achievable.
"""

import sys

import torch

BF16_PEAK_TF = 2500.0
HBM_SPEC_GBS = 8000.0
HBM_ACHIEVABLE_GBS = 6300.0


def trace_work(arch):
    """Per-image work of one config: list of (kind, flops) + BN elems + params."""
    import os
    os.environ.setdefault("CEREBRO_BACKEND", "torch")
    from ..models import create_model_from_mst
    from ..ops import nn as P
    from ..runtime import Arena
    from ..ops.backend import set_backend
    set_backend("torch")
    net = create_model_from_mst({"model": arch})
    arena = Arena(net.layout, 1, "cpu", torch.float32)
    arena.init_model(0, 1)
    net.bind(arena)
    rec = {"gemm": [], "bn_elems": 0}
    first = [True]

    def conv_like(x, wshape, y, groups=1):
        # y: [B, Ho, Wo, Cout] (NHWC packed, G=1); wshape (cout, kh, kw, cin/groups)
        cout = wshape[0]
        k = 1
        for d in wshape[1:]:
            k *= d
        m = y.numel() // cout
        f = 2.0 * m * cout * k
        rec["gemm"].append((f, not first[0]))
        first[0] = False

    orig = {}

    def wrap(name, fn):
        orig[name] = getattr(P, name)

        def w(*a, **k):
            out = orig[name](*a, **k)
            fn(out, *a, **k)
            return out
        setattr(P, name, w)

    wrap("conv2d", lambda y, x, wref, *a, **k: conv_like(x, wref.spec.shape, y))
    wrap("conv2d_bias_act", lambda y, x, wref, *a, **k: conv_like(x, wref.spec.shape, y))
    wrap("grouped_conv2d", lambda y, x, wref, *a, **k: conv_like(x, wref.spec.shape, y))
    wrap("dwconv2d", lambda y, x, wref, *a, **k: conv_like(x, (y.shape[-1],) +
                                                          tuple(wref.spec.shape[1:]) + (1,), y))
    wrap("linear", lambda y, x, wref, *a, **k: conv_like(x, wref.spec.shape, y))

    def bn_cnt(y, x, *a, **k):
        rec["bn_elems"] += x.numel()
    wrap("bn_act", bn_cnt)
    try:
        shape = (1, net.input_hw, net.input_hw, net.input_c)
        with torch.no_grad():
            net.forward(torch.rand(shape), False)
    finally:
        for n, f in orig.items():
            setattr(P, n, f)
    rec["params"] = net.layout.num_params
    return rec


def roofline_rows(fam_ms, arch, configs, batch, dtype):
    """fam_ms: {family label: ms per step} (tools.prof_summary families)."""
    w = trace_work(arch)
    imgs = configs * batch
    esz = 4 if dtype == "fp32" else 2
    passes = 3 if dtype == "fp32" else 1
    fwd = sum(f for f, _ in w["gemm"]) * imgs
    dgrad = sum(f for f, d in w["gemm"] if d) * imgs
    wgrad = fwd
    bn_bytes = 5.0 * esz * w["bn_elems"] * imgs
    adam_bytes = 32.0 * w["params"] * configs

    def get(sub):
        return sum(v for k, v in fam_ms.items() if sub in k)
    rows = []
    for label, key, work in (("conv/linear fwd", "NT: fwd", fwd),
                             ("conv dgrad", "dgrad", dgrad),
                             ("conv/linear wgrad", "wgrad", wgrad)):
        ms = get(key)
        if ms <= 0:
            continue
        tf = work / (ms * 1e-3) / 1e12
        rows.append((label, ms, "{:.1f} GFLOP".format(work / 1e9),
                     "{:.0f} TF ({:.0f} TF MFMA-issued)".format(tf, tf * passes),
                     "{:.1f}% of {:.0f} TF".format(100.0 * tf * passes / BF16_PEAK_TF,
                                                   BF16_PEAK_TF)))
    for label, key, byt in (("batchnorm", "batchnorm", bn_bytes),
                            ("adam", "adam", adam_bytes)):
        ms = get(key)
        if ms <= 0:
            continue
        gbs = byt / (ms * 1e-3) / 1e9
        rows.append((label, ms, "{:.2f} GB (min traffic)".format(byt / 1e9),
                     "{:.0f} GB/s".format(gbs),
                     "{:.1f}% of {:.0f} GB/s achievable".format(100.0 * gbs / HBM_ACHIEVABLE_GBS,
                                                                HBM_ACHIEVABLE_GBS)))
    total = sum(fam_ms.values())
    step_tf = (fwd + dgrad + wgrad) / (total * 1e-3) / 1e12 if total else 0.0
    return rows, step_tf, total


def roofline_md(fam_ms, arch, configs, batch, dtype):
    rows, step_tf, total = roofline_rows(fam_ms, arch, configs, batch, dtype)
    out = ["## roofline ({} x{} configs, batch {}, {})".format(arch, configs, batch, dtype), "",
           "| family | ms/step | work | achieved | vs peak |", "|---|---:|---:|---:|---:|"]
    for r in rows:
        out.append("| {} | {:.3f} | {} | {} | {} |".format(*r))
    out.append("")
    out.append("Whole step: {:.2f} ms of kernels, {:.0f} TF fp32-equivalent GEMM throughput "
               "(all conv/linear FLOPs / step kernel time).".format(total, step_tf))
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    import argparse
    from .prof_summary import family_ms
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--configs", type=int, default=8)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--last-steps", type=int, default=10)
    a = ap.parse_args()
    fam = family_ms(a.path, a.last_steps)
    sys.stdout.write(roofline_md(fam, a.model, a.configs, a.batch, a.dtype))
