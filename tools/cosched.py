#!/usr/bin/env python3
"""Co-scheduling of the fold with the transport on one GPU: P in-process ranks on cuda:0, a
width-P tree in the direct forms, the reduce stream limited to `reduce_cus` CUs (ftar_comm_set_reduce_cus)
so the transport's copy kernels on the comm stream keep free CUs while a piece's fold runs.

On one GPU the local transport's transfers are device copies (blit kernels) -- the stand-in for RCCL's p2p
kernels of a real node, which need CUs the same way.  Prints one JSON line per (reduce_cus, chunk): ms per
call (best and median of --iters, each call synchronised) and whether the output equals the all-CU run's.

    python tools/cosched.py --ranks 8 --elements 67108864
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "allreduce-over-mpi_amd")]

ap = argparse.ArgumentParser()
ap.add_argument("--ranks", type=int, default=8)
ap.add_argument("--topo", default=None)
ap.add_argument("--elements", type=int, default=1 << 26)
ap.add_argument("--iters", type=int, default=8)
ap.add_argument("--cus", default="0,240,224,192,160,128")
ap.add_argument("--chunks", default="4194304,16777216")
a = ap.parse_args()

import torch  # noqa: E402
import ftar  # noqa: E402

torch.cuda.set_device(0)
P, n = a.ranks, a.elements
g = ftar.Comm.init_local(P)
g.set_allgather("direct")
g.set_reduce_scatter("direct")
topo = a.topo or str(P)
gen = torch.Generator(device="cuda").manual_seed(5)
xs = [torch.rand(n, device="cuda", generator=gen) * 2 - 1 for _ in range(P)]
ys = [torch.empty_like(x) for x in xs]
ref = None
for chunk in [int(c) for c in a.chunks.split(",")]:
    g.set_chunk_bytes(chunk)
    for cus in [int(c) for c in a.cus.split(",")]:
        g.set_reduce_cus(cus)
        g.allreduce(xs, ys, n, "f32", "sum", topo_=topo)   # warm-up (and growth)
        torch.cuda.synchronize()
        same = True
        if ref is None:
            ref = [y.clone() for y in ys]
        else:
            same = all(torch.equal(y, r) for y, r in zip(ys, ref))
        ts = []
        for _ in range(a.iters):
            t0 = time.perf_counter()
            g.allreduce(xs, ys, n, "f32", "sum", topo_=topo)
            torch.cuda.synchronize()   # the group call returns once enqueued
            ts.append((time.perf_counter() - t0) * 1e3)
        print(json.dumps({"ranks": P, "topo": topo, "elements": n, "chunk_bytes": chunk,
                          "reduce_cus": cus or "all", "ms_best": round(min(ts), 3),
                          "ms_median": round(statistics.median(ts), 3), "same_bits_as_all_cus": same}), flush=True)
g.set_reduce_cus(0)
g.destroy()
