"""Run one packed conv shape's fwd / dgrad / wgrad a few times (profiling target).

    python scripts/dev/conv_one.py --shape 32,7,7,256,256,3,1,1 --G 8 --iters 20
"""

import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import argparse

import torch

from cerebro_ds_kpgi_amd.ops import backend
from cerebro_ds_kpgi_amd.tools.bench_conv import bench_shape


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="32,7,7,256,256,3,1,1")
    ap.add_argument("--G", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--miopen", action="store_true", help="also time MIOpen")
    a = ap.parse_args(argv)
    backend.set_backend("hip")
    shape = tuple(int(v) for v in a.shape.split(","))
    r = bench_shape(shape, a.G, a.iters, torch.float32 if a.dtype == "fp32" else torch.bfloat16,
                    miopen=a.miopen)
    torch.cuda.synchronize()
    print(shape, {k: round(v, 1) for k, v in r["tflops"].items()})


if __name__ == "__main__":
    main()
