"""Per-layer conv benchmark: our MFMA implicit-GEMM kernels vs MIOpen (PyTorch
grouped conv on channels-last tensors), for every unique ResNet-50@112 conv
shape of the packed G-config model, in bf16 or fp32 (the reference
precision: 3-pass split-bf16 MFMA on our side, MIOpen's fp32 kernels on
the other).

    python -m cerebro_ds_kpgi_amd.tools.bench_conv --G 8 --B 32 [--dtype fp32] [--json out.json]

Reports time and TFLOP/s for fwd, dgrad and wgrad per shape, plus totals
weighted by how often each shape occurs in ResNet-50.
"""

import argparse
import collections
import json

import torch
import torch.nn.functional as F

from ..models import create_model_from_mst
from ..ops import _hip, backend
from ..runtime.arena import Arena, ModelLayout, ParamRef, ParamSpec


def resnet50_shapes(B, hw=112):
    net = create_model_from_mst({"model": "resnet50"})
    shapes = collections.Counter()
    h = hw
    # stem
    shapes[(B, h, h, 3, 64, 7, 2, 3)] += 1
    h = (h + 6 - 7) // 2 + 1
    h = (h + 2 - 3) // 2 + 1
    cin = 64
    for blk in net.blocks:
        c1 = blk["c1"]
        hin = h
        s = c1.stride
        shapes[(B, hin, hin, c1.cin, c1.cout, c1.k, s, c1.pad)] += 1
        h2 = (hin + 2 * c1.pad - c1.k) // s + 1
        c2 = blk["c2"]
        shapes[(B, h2, h2, c2.cin, c2.cout, c2.k, 1, c2.pad)] += 1
        c3 = blk["c3"]
        shapes[(B, h2, h2, c3.cin, c3.cout, 1, 1, 0)] += 1
        if "cs" in blk:
            cs = blk["cs"]
            shapes[(B, hin, hin, cs.cin, cs.cout, 1, cs.stride, 0)] += 1
        h = h2
    return shapes


def _time(fn, iters):
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def bench_shape(shape, G, iters, dtype=torch.bfloat16, miopen=True):
    B, H, W, cin, cout, k, st, pad = shape
    spec = ParamSpec("w", (cout, k, k, cin), "weight", fan_in=k * k * cin)
    lay = ModelLayout([spec])
    a = Arena(lay, G, "cuda", dtype)
    for g in range(G):
        a.init_model(g, g)
    ref = ParamRef(a, spec)
    x = torch.randn(B, H, W, G * cin, device="cuda").to(dtype)
    Ho = (H + 2 * pad - k) // st + 1
    Wo = (W + 2 * pad - k) // st + 1
    dy = torch.randn(B, Ho, Wo, G * cout, device="cuda").to(dtype)
    flops = 2.0 * B * Ho * Wo * cout * k * k * cin * G
    out = {}
    out["hip_fwd"] = _time(lambda: _hip.conv2d_fwd(x, ref, st, pad), iters)
    out["hip_dgrad"] = _time(lambda: _hip.conv2d_dgrad(dy, ref, x.shape, st, pad), iters)
    out["hip_wgrad"] = _time(lambda: _hip.conv2d_wgrad(x, dy, ref, st, pad), iters)
    if not miopen:
        out["tflops"] = {kk: flops / (v * 1e-3) / 1e12 for kk, v in out.items()}
        out["gflop"] = flops / 1e9
        return out
    w = ref.work().permute(0, 1, 4, 2, 3).reshape(G * cout, cin, k, k).contiguous(
        memory_format=torch.channels_last)
    xn = x.permute(0, 3, 1, 2)
    dyn = dy.permute(0, 3, 1, 2)
    out["miopen_fwd"] = _time(lambda: F.conv2d(xn, w, None, st, pad, 1, G), iters)
    out["miopen_dgrad"] = _time(
        lambda: torch.nn.grad.conv2d_input(xn.shape, w, dyn, st, pad, 1, G), iters)
    out["miopen_wgrad"] = _time(
        lambda: torch.nn.grad.conv2d_weight(xn, w.shape, dyn, st, pad, 1, G), iters)
    out["tflops"] = {kk: flops / (v * 1e-3) / 1e12 for kk, v in out.items()}
    out["gflop"] = flops / 1e9
    return out


VARIANTS = {0: "reg64", 1: "reg128", 2: "reg128x64", 3: "dma64", 4: "dma128", 5: "dma128x64"}


def _vname(v):
    """conv.hip variant id -> name (fp32 forward: 12-23 = 32x32x16-MFMA twins)."""
    w, v = ("w", v - 12) if v >= 12 else ("", v)
    return "{}{}{}{}".format(w, "sk" if v >= 6 else "", "dma" if (v // 3) & 1 else "reg",
                             ("64", "128", "128x64")[v % 3])


def sweep(shapes, G, iters, dtype=torch.bfloat16, ops_sel=(0, 1, 2)):
    """Time every kernel variant of every op on every shape (HIP only).
    Returns the rows plus, per op, the count-weighted step time of the best
    variant per shape among ids < 12 ("narrow") and among all ids."""
    out = []
    tot = collections.defaultdict(float)
    for shape, count in shapes.items():
        B, H, W, cin, cout, k, st, pad = shape
        if cin % 8:
            continue
        spec = ParamSpec("w", (cout, k, k, cin), "weight", fan_in=k * k * cin)
        a = Arena(ModelLayout([spec]), G, "cuda", dtype)
        for g in range(G):
            a.init_model(g, g)
        ref = ParamRef(a, spec)
        x = torch.randn(B, H, W, G * cin, device="cuda").to(dtype)
        Ho = (H + 2 * pad - k) // st + 1
        Wo = (W + 2 * pad - k) // st + 1
        dy = torch.randn(B, Ho, Wo, G * cout, device="cuda").to(dtype)
        row = {"shape": shape, "count": count}
        ops = {0: lambda: _hip.conv2d_fwd(x, ref, st, pad),
               1: lambda: _hip.conv2d_dgrad(dy, ref, x.shape, st, pad),
               2: lambda: _hip.conv2d_wgrad(x, dy, ref, st, pad)}
        for op in ops_sel:
            fn = ops[op]
            vs = _hip.FP32_VARIANTS[op] if dtype == torch.float32 else tuple(VARIANTS)
            times = {}
            for v in vs:
                _hip.conv_set_variant(op, v)
                times[v] = _time(fn, iters)
                row["{}:{}".format(op, _vname(v))] = times[v]
            _hip.conv_set_variant(op, -1)
            narrow = min(t for v, t in times.items() if v < 12)
            tot["{}:narrow".format(op)] += count * narrow
            tot["{}:all".format(op)] += count * min(times.values())
            row["{}:best".format(op)] = _vname(min(times, key=times.get))
        out.append(row)
        print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in row.items()}),
              flush=True)
    print("SWEEP_TOTAL_MS", json.dumps({k: round(v, 3) for k, v in tot.items()}), flush=True)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--G", type=int, default=8)
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--json", default="")
    ap.add_argument("--sweep", action="store_true", help="time every kernel variant per shape")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--ops", default="0,1,2", help="ops to sweep: 0 fwd, 1 dgrad, 2 wgrad")
    ap.add_argument("--no_miopen", action="store_true", help="time our kernels only")
    a = ap.parse_args(argv)
    dtype = torch.float32 if a.dtype == "fp32" else torch.bfloat16
    backend.set_backend("hip")
    if a.sweep:
        rows = sweep(resnet50_shapes(a.B), a.G, a.iters, dtype,
                     tuple(int(o) for o in a.ops.split(",")))
        if a.json:
            with open(a.json, "w") as f:
                json.dump(rows, f, indent=1, default=str)
        return
    rows = []
    tot = collections.defaultdict(float)
    for shape, count in resnet50_shapes(a.B).items():
        r = bench_shape(shape, a.G, a.iters, dtype, miopen=not a.no_miopen)
        for kk in ("miopen_fwd", "miopen_dgrad", "miopen_wgrad"):
            r.setdefault(kk, float("nan"))
            r["tflops"].setdefault(kk, float("nan"))
        r["shape"] = shape
        r["count"] = count
        rows.append(r)
        for kk in ("hip_fwd", "hip_dgrad", "hip_wgrad", "miopen_fwd", "miopen_dgrad", "miopen_wgrad"):
            tot[kk] += count * r[kk]
        tot["gflop"] += count * r["gflop"]
        print("{:<34} x{:<2} {:7.2f} GF | fwd {:6.1f} vs {:6.1f} TF | dgrad {:6.1f} vs {:6.1f} | "
              "wgrad {:6.1f} vs {:6.1f}".format(
                  str(shape), count, r["gflop"], r["tflops"]["hip_fwd"], r["tflops"]["miopen_fwd"],
                  r["tflops"]["hip_dgrad"], r["tflops"]["miopen_dgrad"],
                  r["tflops"]["hip_wgrad"], r["tflops"]["miopen_wgrad"]), flush=True)
    hip = tot["hip_fwd"] + tot["hip_dgrad"] + tot["hip_wgrad"]
    mio = tot["miopen_fwd"] + tot["miopen_dgrad"] + tot["miopen_wgrad"]
    summary = {"G": a.G, "B": a.B, "dtype": a.dtype, "hip_ms_per_step": hip, "miopen_ms_per_step": mio,
               "hip_tflops": 3 * tot["gflop"] / hip, "miopen_tflops": 3 * tot["gflop"] / mio,
               "fwd_ms": {"hip": tot["hip_fwd"], "miopen": tot["miopen_fwd"]},
               "dgrad_ms": {"hip": tot["hip_dgrad"], "miopen": tot["miopen_dgrad"]},
               "wgrad_ms": {"hip": tot["hip_wgrad"], "miopen": tot["miopen_wgrad"]}}
    print("TOTAL", json.dumps(summary))
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"summary": summary, "rows": rows}, f, indent=1, default=str)


if __name__ == "__main__":
    main()
