#!/usr/bin/env python3
"""Interleaved A/B of reduce-kernel variants in ONE process (guide rule 24).

    python tools/kbench.py [--elements N] [--rounds R] [--variants 0,1,..] [--ks 2,4,8] [--dtypes f32,bf16]
Each variant = (vectors/lane, nt loads, nt stores, workgroup size, grid cap),
see ftar_debug_reduce_variant in csrc/bench_kernels.hip (libftar_bench.so).  Prints median/min
kernel time and GB/s ((k+1)*n*esz bytes) per (dtype, k, variant), plus a
device-to-device copy as a reference point.  Every variant's output is
compared with variant 0's.
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
ap.add_argument("--elements", type=int, default=1 << 26)
ap.add_argument("--rounds", type=int, default=10)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--variants", default="0,1,2,3,4,5,6,7,8,9,10,11")
ap.add_argument("--ks", default="2,4,8")
ap.add_argument("--dtypes", default="f32,bf16")
ap.add_argument("--shapes", default="", help='nested folds instead of variants, e.g. "8;2,4;2,2,2" ("8" = flat)')
a = ap.parse_args()
lib = ftar.bench_lib()
lib.ftar_debug_reduce_variant.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                                          ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
dev = torch.device("cuda:0")
n = a.elements
variants = [int(v) for v in a.variants.split(",")]
ks = [int(k) for k in a.ks.split(",")]
dts = a.dtypes.split(",")
tdt = {"f32": torch.float32, "bf16": torch.bfloat16}
srcs = {d: [(torch.rand(n, device=dev) * 2 - 1).to(tdt[d]) for _ in range(max(ks))] for d in dts}
dst = {d: torch.empty(n, device=dev, dtype=tdt[d]) for d in dts}
ref = {}
stream = torch.cuda.current_stream()
res = {}
for r in range(a.rounds):
    for d in dts:
        esz = 4 if d == "f32" else 2
        for k in ks:
            arr = (ctypes.c_void_p * k)(*[s.data_ptr() for s in srcs[d][:k]])
            for v in variants:
                st = lib.ftar_debug_reduce_variant(v, ftar.DTYPE[d], arr, k, dst[d].data_ptr(), n, stream.cuda_stream)
                assert st == 0, (d, k, v, st)
                if r == 0:
                    torch.cuda.synchronize()
                    if v == variants[0]:
                        ref[(d, k)] = dst[d].clone()
                    else:
                        assert torch.equal(dst[d].view(torch.int16 if esz == 2 else torch.int32),
                                           ref[(d, k)].view(torch.int16 if esz == 2 else torch.int32)), (d, k, v)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(a.reps):
                    lib.ftar_debug_reduce_variant(v, ftar.DTYPE[d], arr, k, dst[d].data_ptr(), n, stream.cuda_stream)
                e1.record(stream)
                torch.cuda.synchronize()
                res.setdefault((d, k, v), []).append(e0.elapsed_time(e1) / a.reps)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    x = srcs[dts[0]][0]
    y = dst[dts[0]]
    e0.record(stream)
    for _ in range(a.reps):
        y.copy_(x)
    e1.record(stream)
    torch.cuda.synchronize()
    res.setdefault(("copy", 0, 0), []).append(e0.elapsed_time(e1) / a.reps)

if a.shapes:  # flat k-way (ftar_reduce) vs nested folds (ftar_reduce_nested) of the same k, interleaved
    shapes = [[int(w) for w in sh.split(",")] for sh in a.shapes.split(";")]
    res = {}
    kmax = max(int(torch.tensor(sh).prod()) for sh in shapes)
    for d in dts:
        while len(srcs[d]) < kmax:
            srcs[d].append((torch.rand(n, device=dev) * 2 - 1).to(tdt[d]))
    for r in range(a.rounds):
        for d in dts:
            for sh in shapes:
                k = int(torch.tensor(sh).prod())
                ptrs = [s_.data_ptr() for s_ in srcs[d][:k]]
                call = lambda: ftar.reduce(ptrs, dst[d].data_ptr(), n, d, "sum", stream=stream.cuda_stream,
                                           shape=sh if len(sh) > 1 else None)
                call()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(a.reps):
                    call()
                e1.record(stream)
                torch.cuda.synchronize()
                res.setdefault((d, k, ",".join(map(str, sh))), []).append(e0.elapsed_time(e1) / a.reps)

for (d, k, v), ts in sorted(res.items(), key=lambda kv: str(kv[0])):
    esz = 4 if d in ("f32", "copy") else 2
    byts = (2 if d == "copy" else k + 1) * n * esz
    med, mn = statistics.median(ts), min(ts)
    print(json.dumps({"dtype": d, "k": k, "variant": v, "ms_med": round(med, 4), "ms_min": round(mn, 4),
                      "GBps_med": round(byts / med / 1e6, 1), "GBps_max": round(byts / mn / 1e6, 1)}))
