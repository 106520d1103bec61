#!/usr/bin/env python3
"""Host-memory end-to-end rate of the AllReduce path (DESIGN.md §Host path).

The reference's buffers live in host memory (MPI send/recv buffers,
benchmark.cpp:125-131).  Measured on one MI355X: pinned H2D and D2H of one
bucket alone and both directions at once, the device AllReduce of P
in-process ranks, the serial host->host call (H2D, AllReduce, D2H), and
ftar_allreduce_host (H2D / exchange / D2H pipelined per piece; the
MPI_Allreduce_FT path) at several piece sizes.  With P ranks on one GPU all
ranks share this GPU's PCIe link, so pcie_GBps = P * bucket / t per direction.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "allreduce-over-mpi_amd"))
import torch  # noqa: E402
import ftar  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best


import argparse  # noqa: E402
ap = argparse.ArgumentParser()
ap.add_argument("--sizes", default="20,26,28", help="log2 elements per bucket")
ap.add_argument("--chunks", default="1024,16,4,1", help="host piece sizes in MiB (1024 = one piece: serial)")
ap.add_argument("--ranks", default="2,8")
a = ap.parse_args()
dev = torch.device("cuda:0")
out = []
for n in [1 << int(x) for x in a.sizes.split(",")]:
    nbytes = n * 4
    h = torch.rand(n).pin_memory()
    hp = torch.empty(n).pin_memory()
    hpg = torch.empty(n)                # pageable
    d = torch.empty(n, device=dev)
    t_h2d = timeit(lambda: d.copy_(h, non_blocking=True))
    t_d2h = timeit(lambda: hp.copy_(d, non_blocking=True))
    t_d2h_pageable = timeit(lambda: hpg.copy_(d))
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    d2 = torch.empty(n, device=dev)

    def both():
        with torch.cuda.stream(s1):
            d.copy_(h, non_blocking=True)
        with torch.cuda.stream(s2):
            hp.copy_(d2, non_blocking=True)
    t_both = timeit(both)
    row = {"bytes": nbytes, "h2d_GBps": round(nbytes / t_h2d / 1e9, 2), "d2h_GBps": round(nbytes / t_d2h / 1e9, 2),
           "d2h_pageable_GBps": round(nbytes / t_d2h_pageable / 1e9, 2),
           "h2d_and_d2h_concurrent_GBps_per_dir": round(nbytes / t_both / 1e9, 2)}
    for P in [int(x) for x in a.ranks.split(",")]:
        topo = str(P)
        if n > (1 << 26) and P > 2:
            continue
        g = ftar.Comm.init_local(P)
        ds = [torch.rand(n, device=dev) for _ in range(P)]
        hs = [torch.rand(n).pin_memory() for _ in range(P)]
        t_dev = timeit(lambda: g.allreduce(None, ds, n, "f32", topo_=topo))

        def e2e():
            for r in range(P):
                ds[r].copy_(hs[r], non_blocking=True)
            g.allreduce(None, ds, n, "f32", topo_=topo, streams=[torch.cuda.current_stream()] * P)
            for r in range(P):
                hs[r].copy_(ds[r], non_blocking=True)
        t_e2e = timeit(e2e)
        row[f"P{P}_device_ms"] = round(t_dev * 1e3, 3)
        row[f"P{P}_host_e2e_ms"] = round(t_e2e * 1e3, 3)
        for chunk in [int(c) << 20 for c in a.chunks.split(",")]:
            g.set_host_chunk_bytes(chunk)
            t_h = timeit(lambda: g.allreduce(None, hs, n, "f32", topo_=topo, host=True))
            row[f"P{P}_host_pipelined_c{chunk >> 20}MiB_ms"] = round(t_h * 1e3, 3)
            row[f"P{P}_host_pipelined_c{chunk >> 20}MiB_pcie_GBps"] = round(P * nbytes / t_h / 1e9, 2)
        g.set_host_chunk_bytes(0)
        g.destroy()
        del ds, hs
    out.append(row)
    print(json.dumps(row), flush=True)
