"""Measure the per-kernel floor of a HIP-graph replay on this GPU.

    python scripts/dev/launch_floor.py [--n 300]

Captures ``n`` dependent tiny kernels (one-block in-place adds, and
256-block ones) in a graph and reports replay wall time per kernel; then
the same ``n`` kernels split over two streams (fork/join inside the graph)
to see how much of the floor two independent chains overlap.  This is the
question behind the one-config ResNet-50 step (~300 kernels per step).
"""

import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import argparse
import json
import time

import torch


def _time_graph(fn, reps=50):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=300)
    a = ap.parse_args()
    n = a.n
    dev = torch.device("cuda")
    small = torch.zeros(64, device=dev)
    wide = torch.zeros(256 * 256 * 4, device=dev)     # 256 blocks of 256 threads x 4
    side = torch.cuda.Stream()
    res = {}

    def chain(t, k):
        for _ in range(k):
            t.add_(1.0)

    res["one_block_us"] = 1e6 * _time_graph(lambda: chain(small, n)) / n
    res["256_block_us"] = 1e6 * _time_graph(lambda: chain(wide, n)) / n
    small2 = torch.zeros(64, device=dev)
    wide2 = torch.zeros_like(wide)

    def two(t1, t2):
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            chain(t2, n // 2)
        chain(t1, n // 2)
        cur.wait_stream(side)

    res["one_block_2streams_us"] = 1e6 * _time_graph(lambda: two(small, small2)) / n
    res["256_block_2streams_us"] = 1e6 * _time_graph(lambda: two(wide, wide2)) / n
    res["n"] = n
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
