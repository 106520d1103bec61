#!/usr/bin/env python3
"""PCIe piece rates for the host path: a 256 MiB bucket moved in pieces of
1..64 MiB, one stream, by the runtime's copies (hipMemcpyAsync: SDMA for H2D, blit kernels for D2H on this
image) and by ftar's own streaming copy kernel (ftar_reduce with k = 1) reading or writing the pinned host
buffer directly over PCIe; then both directions at once on two streams.  Prints one JSON line per case."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "allreduce-over-mpi_amd"))
import torch  # noqa: E402

import ftar  # noqa: E402

TOTAL = 256 << 20
N = TOTAL // 4
dev = torch.device("cuda", 0)
x = torch.rand(N, device=dev)
y = torch.empty_like(x)
hx = torch.rand(N).pin_memory()
hy = torch.empty(N).pin_memory()
s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()


def pieces(piece_mib):
    m = (piece_mib << 20) // 4
    return [(i, min(m, N - i)) for i in range(0, N, m)]


def d2h(method, piece_mib, s):
    for i, m in pieces(piece_mib):
        if method == "memcpy":
            with torch.cuda.stream(s):
                hy[i:i + m].copy_(x[i:i + m], non_blocking=True)
        else:
            ftar.reduce([x.data_ptr() + 4 * i], hy.data_ptr() + 4 * i, m, "f32", "sum", stream=s)


def h2d(method, piece_mib, s):
    for i, m in pieces(piece_mib):
        if method == "memcpy":
            with torch.cuda.stream(s):
                y[i:i + m].copy_(hx[i:i + m], non_blocking=True)
        else:
            ftar.reduce([hx.data_ptr() + 4 * i], y.data_ptr() + 4 * i, m, "f32", "sum", stream=s)


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best


for piece in (1, 4, 16, 64):
    for method in ("memcpy", "kernel"):
        td = timed(lambda: d2h(method, piece, s0))
        assert torch.equal(hy, x.cpu()), ("d2h", method, piece)
        th = timed(lambda: h2d(method, piece, s0))
        assert torch.equal(y.cpu(), hx), ("h2d", method, piece)
        tb = timed(lambda: (h2d(method, piece, s1), d2h(method, piece, s0)))
        print(json.dumps({"piece_MiB": piece, "method": method, "d2h_GBps": round(TOTAL / td / 1e9, 1),
                          "h2d_GBps": round(TOTAL / th / 1e9, 1),
                          "both_GBps_each": round(TOTAL / tb / 1e9, 1)}), flush=True)
