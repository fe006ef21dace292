"""Time the BatchNorm apply kernels of one packed layer shape (fp32, HIP).

    python scripts/dev/bn_one.py --rows 1568 --C 256 --G 1 --iters 200

Times, per launch (CUDA events around ``iters`` back-to-back launches; and
the same launches replayed from a HIP graph, the training step's form):

* fwd: ``bn_act_fwd_train_part`` from fp64 conv-epilogue slabs (the fold
  kernel: finalize + running statistics + apply), plain and HL output,
  with and without a residual;
* bwd: ``bn_act_bwd`` from dgrad-epilogue slabs (mask from z: YM_Z, and
  the residual-join form: YM_Y).

Prints one JSON line per case: us per launch eager / graph and GB/s.
"""

import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import argparse
import json

import torch

from cerebro_ds_kpgi_amd.ops import _hip, backend
from cerebro_ds_kpgi_amd.runtime.arena import Arena, ModelLayout, ParamRef, ParamSpec

SLAB_F64 = 1 << 24


def _refs(C, G):
    specs = [ParamSpec("g", (C,), "gamma"), ParamSpec("b", (C,), "beta"),
             ParamSpec("rm", (C,), "running_mean"), ParamSpec("rv", (C,), "running_var")]
    a = Arena(ModelLayout(specs), G, "cuda", torch.float32)
    for g in range(G):
        a.init_model(g, g)
    return a, {s.name: ParamRef(a, s) for s in specs}


def _slabs(t, n):
    """fp64 slab partials [n][2][C] of rows of t (what a conv epilogue makes)."""
    C = t.shape[-1]
    x = t.reshape(-1, C).double()
    out = torch.zeros(n, 2, C, dtype=torch.float64, device=t.device)
    for i, chunk in enumerate(x.chunk(n)):
        out[i, 0] = chunk.sum(0)
        out[i, 1] = (chunk * chunk).sum(0)
    return out.view(torch.float32).reshape(-1), n | SLAB_F64


def _time(fn, iters, graph):
    fn()
    torch.cuda.synchronize()
    if graph:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(iters):
                fn()
        g.replay()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
    else:
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
    e.synchronize()
    return 1000.0 * s.elapsed_time(e) / iters


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1568)
    ap.add_argument("--C", type=int, default=256, help="channels per config")
    ap.add_argument("--G", type=int, default=1)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--nslab", type=int, default=8)
    a = ap.parse_args(argv)
    backend.set_backend("hip")
    C, G, M = a.C, a.G, a.rows
    arena, r = _refs(C, G)
    z = torch.randn(M, G * C, device="cuda")
    res = torch.randn(M, G * C, device="cuda")
    dy = torch.randn(M, G * C, device="cuda")
    part, nslab = _slabs(z, min(a.nslab, M // 64 or 1))
    mean = z.mean(0)
    invstd = torch.rsqrt(z.var(0, unbiased=False) + 1e-5)
    y = torch.relu(z)
    bpart, bnslab = _slabs(dy, min(a.nslab, M // 64 or 1))
    nbytes = M * G * C * 4

    cases = {
        "fwd": (lambda: _hip.bn_act_fwd_train_part(z, None, r["g"], r["b"], r["rm"], r["rv"], 1,
                                                   0.1, 1e-5, part, nslab), 2),
        "fwd_hl": (lambda: _hip.bn_act_fwd_train_part(z, None, r["g"], r["b"], r["rm"], r["rv"],
                                                      1, 0.1, 1e-5, part, nslab, hl_out=True), 2),
        "fwd_res": (lambda: _hip.bn_act_fwd_train_part(z, res, r["g"], r["b"], r["rm"], r["rv"],
                                                       1, 0.1, 1e-5, part, nslab), 3),
        "bwd_zmask_hl": (lambda: _hip.bn_act_bwd(dy, z, y, mean, invstd, r["g"], r["b"], 1, False,
                                                 part=bpart, nslab=bnslab, hl_out=True), 3),
        "bwd_res": (lambda: _hip.bn_act_bwd(dy, z, y, mean, invstd, r["g"], r["b"], 1, True,
                                            part=bpart, nslab=bnslab), 5),
    }
    for name, (fn, tensors) in cases.items():
        t_e = _time(fn, a.iters, False)
        t_g = _time(fn, a.iters, True)
        print(json.dumps({"case": name, "rows": M, "C": C, "G": G, "us_eager": round(t_e, 2),
                          "us_graph": round(t_g, 2),
                          "GBps_graph": round(tensors * nbytes / t_g / 1e3, 1)}))


if __name__ == "__main__":
    main()
