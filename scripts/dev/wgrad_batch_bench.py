"""Isolated timing of the batched fp32 weight gradients of one ResNet-50 step.

    python scripts/dev/wgrad_batch_bench.py --G 8 [--variants 0,1,2,12,13,14]

Queues the weight gradient of every aligned ResNet-50 conv (bs 32, 112x112,
``resnet50_shapes``) inside one ``streams.deferred_wgrad`` block and times the
flush, which is what the training step launches at the end of backward.  It
does this for each batch kernel variant (``CER_WGB_VARIANT`` ids) and rows
per split (``CER_WGB_ROWS``).  As a bound, it also times the per-layer
autotuned unbatched kernels (``cer_conv_wgrad``).  Prints one JSON line per
configuration: ms per flush and the fp32-equivalent TFLOP/s over the
step's wgrad FLOPs.  The stem (Cin = 3) takes its own path and is left out.
"""

import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import argparse
import json
import statistics

import torch

from cerebro_ds_kpgi_amd.ops import _hip, backend, streams
from cerebro_ds_kpgi_amd.runtime.arena import Arena, ModelLayout, ParamRef, ParamSpec
from cerebro_ds_kpgi_amd.tools.bench_conv import resnet50_shapes


def _layers(G, B, dtype=torch.float32):
    out = []
    flops = 0.0
    for shape, count in resnet50_shapes(B).items():
        b, H, W, cin, cout, k, st, pad = shape
        if cin % 8:
            continue
        Ho = (H + 2 * pad - k) // st + 1
        Wo = (W + 2 * pad - k) // st + 1
        for _ in range(count):
            spec = ParamSpec("w", (cout, k, k, cin), "weight", fan_in=k * k * cin)
            a = Arena(ModelLayout([spec]), G, "cuda", dtype)
            ref = ParamRef(a, spec)
            x = torch.randn(b, H, W, G * cin, device="cuda", dtype=dtype)
            dy = torch.randn(b, Ho, Wo, G * cout, device="cuda", dtype=dtype)
            out.append((x, dy, ref, st, pad))
            flops += 2.0 * b * Ho * Wo * cout * k * k * cin * G
    return out, flops


def _time(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return statistics.median(ts)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--G", type=int, default=8)
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--variants", default="0,1,2,12,13,14")
    ap.add_argument("--rows", default="0")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args(argv)
    backend.set_backend("hip")
    layers, flops = _layers(a.G, a.B)

    def batched():
        with streams.deferred_wgrad():
            for x, dy, ref, st, pad in layers:
                _hip.conv2d_wgrad(x, dy, ref, st, pad)

    keep = streams._BATCH_VARIANT
    for rows in (int(r) for r in a.rows.split(",")):
        streams.set_batch_rows(rows)
        for v in (int(s) for s in a.variants.split(",")):
            streams.set_batch_variant(v)
            ms = _time(batched, a.reps)
            print(json.dumps({"G": a.G, "mode": "batched", "variant": v,
                              "rows": rows, "layers": len(layers), "ms": round(ms, 3),
                              "tflops": round(flops / (ms * 1e-3) / 1e12, 1)}), flush=True)
    streams.set_batch_variant(keep)
    streams.set_batch_rows(0)

    def unbatched():
        for x, dy, ref, st, pad in layers:
            _hip.conv2d_wgrad(x, dy, ref, st, pad)
    ms = _time(unbatched, a.reps)
    print(json.dumps({"G": a.G, "mode": "per-layer autotuned", "layers": len(layers),
                      "ms": round(ms, 3), "tflops": round(flops / (ms * 1e-3) / 1e12, 1)}),
          flush=True)


if __name__ == "__main__":
    main()
