#!/usr/bin/env python3
"""Drive the engine for a timeline: P in-process ranks on cuda:0, one topology.

    rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d OUT -o run -- \
        python3 tools/engine_trace.py --ranks 8 --topo 8 --elements 67108864
then `python tools/engine_trace.py --analyze OUT/run_kernel_trace.csv OUT/run_memory_copy_trace.csv`
reports how much reduce-kernel time overlaps the transfers (copies), and per
copy direction the busy time and how much host->device and device->host
copies overlap each other (--host: ftar_allreduce_host on pinned buffers).
"""
import argparse
import csv
import json
import os
import sys

ap = argparse.ArgumentParser()
ap.add_argument("--ranks", type=int, default=8)
ap.add_argument("--topo", default="8")
ap.add_argument("--elements", type=int, default=1 << 26)
ap.add_argument("--chunk-bytes", type=int, default=16 << 20)
ap.add_argument("--iters", type=int, default=3)
ap.add_argument("--host", action="store_true", help="host buffers (ftar_allreduce_host)")
ap.add_argument("--host-chunk-bytes", type=int, default=0)
ap.add_argument("--analyze", nargs=2, metavar=("KERNEL_CSV", "COPY_CSV"))
a = ap.parse_args()


def intervals(path, pred, name_key):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if pred(r.get(name_key, "")):
                out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return sorted(out)


def union(iv):
    res = []
    for s, e in iv:
        if res and s <= res[-1][1]:
            res[-1][1] = max(res[-1][1], e)
        else:
            res.append([s, e])
    return res


def overlap(a_iv, b_union):
    tot = 0
    j = 0
    for s, e in a_iv:
        for bs, be in b_union:
            lo, hi = max(s, bs), min(e, be)
            if hi > lo:
                tot += hi - lo
    return tot


if a.analyze:
    kcsv, ccsv = a.analyze
    red = intervals(kcsv, lambda n: "reduce_vec_kernel" in n, "Kernel_Name")
    # device copies: copy kernels in the kernel trace and/or SDMA copies in the memory-copy trace
    copies = intervals(kcsv, lambda n: "copyBuffer" in n or "Copy" in n, "Kernel_Name")
    if os.path.exists(ccsv):
        with open(ccsv) as f:
            rows = list(csv.DictReader(f))
        copies += sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
    cu = union(sorted(copies))
    red_t = sum(e - s for s, e in red)
    ov = overlap(red, cu)
    res = {"reduce_kernels": len(red), "reduce_ns": red_t, "copy_ops": len(copies),
           "copy_busy_ns": sum(e - s for s, e in cu), "reduce_overlapped_ns": ov,
           "reduce_overlap_frac": round(ov / red_t, 4) if red_t else None}
    if os.path.exists(ccsv):
        kinds = {}
        for r in rows:
            kinds.setdefault(r.get("Direction", r.get("Operation", "?")), []).append(
                (int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        for kd, iv in kinds.items():
            u = union(sorted(iv))
            res[f"{kd}_ops"] = len(iv)
            res[f"{kd}_busy_ns"] = sum(e - s for s, e in u)
            res[f"{kd}_span_ns"] = u[-1][1] - u[0][0]
        h2d = [k for k in kinds if "HOST_TO_DEVICE" in k.upper()]
        d2h = [k for k in kinds if "DEVICE_TO_HOST" in k.upper()]
        if h2d and d2h:
            uh, ud = union(sorted(kinds[h2d[0]])), union(sorted(kinds[d2h[0]]))
            res["h2d_d2h_overlap_ns"] = overlap([tuple(x) for x in uh], ud)
    print(json.dumps(res))
    sys.exit(0)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "allreduce-over-mpi_amd"))
import torch  # noqa: E402
import ftar  # noqa: E402

g = ftar.Comm.init_local(a.ranks)
g.set_chunk_bytes(a.chunk_bytes)
g.set_host_chunk_bytes(a.host_chunk_bytes)
if a.host:
    bufs = [torch.rand(a.elements).pin_memory() for _ in range(a.ranks)]
else:
    bufs = [torch.rand(a.elements, device="cuda") for _ in range(a.ranks)]
for _ in range(a.iters):
    g.allreduce(None, bufs, a.elements, "f32", topo_=a.topo, host=a.host)
torch.cuda.synchronize()
g.destroy()
print("done")
