#!/usr/bin/env python3
"""Interleaved A/B of reduce-kernel variants in ONE process (guide rule 24).

    python tools/kbench.py [--n 67108864] [--rounds 10] [--variants 0,1,2,...]
Prints per-(k, variant) median/min kernel time and GB/s ((k+1)*n*4 bytes),
plus a device-to-device copy for reference.
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "allreduce-over-mpi_amd"))
import torch  # noqa: E402
import ftar  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1 << 26)
ap.add_argument("--rounds", type=int, default=10)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--variants", default="0,1,2,3,4,5,6,7,8,9,10,11")
ap.add_argument("--ks", default="2,8")
a = ap.parse_args()
lib = ftar.lib()
lib.ftar_debug_reduce_variant.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_void_p,
                                          ctypes.c_size_t, ctypes.c_void_p]
dev = torch.device("cuda:0")
n = a.n
variants = [int(v) for v in a.variants.split(",")]
ks = [int(k) for k in a.ks.split(",")]
srcs = [torch.rand(n, device=dev) * 2 - 1 for _ in range(max(ks))]
dst = torch.empty(n, device=dev)
stream = torch.cuda.current_stream()
res = {}
ref = {}
for k in ks:
    arr = (ctypes.c_void_p * k)(*[s.data_ptr() for s in srcs[:k]])
    ref[k] = sum(srcs[j] for j in range(k)) if k == 2 else None
for r in range(a.rounds):
    for k in ks:
        arr = (ctypes.c_void_p * k)(*[s.data_ptr() for s in srcs[:k]])
        for v in variants:
            st = lib.ftar_debug_reduce_variant(v, arr, k, dst.data_ptr(), n, stream.cuda_stream)
            assert st == 0, (v, st)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.reps):
                lib.ftar_debug_reduce_variant(v, arr, k, dst.data_ptr(), n, stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize()
            res.setdefault((k, v), []).append(e0.elapsed_time(e1) / a.reps)
            if r == 0 and k == 2:
                assert torch.equal(dst, ref[2]), f"variant {v} wrong"
    # copy reference
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(a.reps):
        dst.copy_(srcs[0])
    e1.record(stream)
    torch.cuda.synchronize()
    res.setdefault(("copy", 0), []).append(e0.elapsed_time(e1) / a.reps)

out = []
for (k, v), ts in sorted(res.items(), key=lambda kv: str(kv[0])):
    byts = (2 if k == "copy" else k + 1) * n * 4
    med, mn = statistics.median(ts), min(ts)
    out.append({"k": k, "variant": v, "ms_med": round(med, 4), "ms_min": round(mn, 4),
                "GBps_med": round(byts / med / 1e6, 1), "GBps_max": round(byts / mn / 1e6, 1)})
    print(json.dumps(out[-1]))
