"""Minimal repro: hipMemsetAsync / hipMemcpyAsync (D2D) captured in a HIP
graph, replayed several times.  Each replay: memset(buf, 0) [or copy zeros
into buf] then buf += 1 (a torch kernel).  Correct: buf == 1 after EVERY
replay."""
import ctypes
import sys

import torch

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                               ctypes.c_void_p]
for n in (1 << 10, 1 << 20, 1 << 24):
    for how in ("memset", "memcpy", "torch_zero", "torch_copy"):
        buf = torch.full((n,), 7.0, device="cuda")
        zeros = torch.zeros(n, device="cuda")
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            s = torch.cuda.current_stream().cuda_stream
            if how == "memset":
                assert hip.hipMemsetAsync(buf.data_ptr(), 0, n * 4, s) == 0
            elif how == "memcpy":
                assert hip.hipMemcpyAsync(buf.data_ptr(), zeros.data_ptr(), n * 4, 3, s) == 0
            elif how == "torch_zero":
                buf.zero_()
            else:
                buf.copy_(zeros)
            buf.add_(1.0)
        res = []
        for r in range(4):
            g.replay()
            torch.cuda.synchronize()
            res.append((float(buf.min()), float(buf.max())))
        ok = all(v == (1.0, 1.0) for v in res)
        print("n=%d %-10s %s %s" % (n, how, "OK " if ok else "BAD", res), flush=True)
