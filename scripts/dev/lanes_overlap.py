"""Do HIP graphs replayed on different torch streams overlap on the GPU?

Captures two graphs of small, latency-bound work (chains of 64x64 matmuls
that occupy a few CUs) and times N replays of each: both on one stream,
then one per stream (the async runtime's lanes, async_mop._Lanes).  Prints
one JSON line; an overlap ratio near 2 means the streams ran concurrently.
"""

import json
import time

import torch


def main():
    dev = torch.device("cuda", 0)
    a = torch.randn(64, 64, device=dev)
    graphs = []
    for _ in range(2):
        x = torch.randn(64, 64, device=dev)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                y = x
                for _ in range(50):
                    y = y @ a
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            y = x
            for _ in range(50):
                y = y @ a
        graphs.append(g)
    lanes = [torch.cuda.Stream(), torch.cuda.Stream()]
    N = 40

    def run(streams):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(N):
            for g, st in zip(graphs, streams):
                with torch.cuda.stream(st):
                    g.replay()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    main_s = torch.cuda.current_stream()
    run([main_s, main_s])
    one = min(run([main_s, main_s]) for _ in range(3))
    two = min(run(lanes) for _ in range(3))
    print(json.dumps({"replays_each": N, "one_stream_s": round(one, 4),
                      "two_streams_s": round(two, 4), "overlap_ratio": round(one / two, 2)}))


if __name__ == "__main__":
    main()
