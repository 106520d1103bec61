#!/usr/bin/env python3
"""Reduce-kernel variants with and without the Infinity Cache (MALL) in play.

    python tools/kbench_cold.py [--elements N] [--sets S] [--ks 2,8] [--variants 0,12,...] [--rounds R]

sets = 1 repeats every launch on the same buffers (the reference harness's loop: a 256 MiB destination
rewritten back to back partly stays in the 256 MB MALL, so fewer writes reach HBM); sets = S > 1 rotates
the launches over S disjoint (k sources + destination) sets, so every launch streams cold data from and
to HBM.  Interleaved rounds; prints one JSON line per (sets, k, variant) with the median GB/s of
(k+1)*n*4 algorithmic bytes.
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
ap.add_argument("--sets", default="1,4")
ap.add_argument("--ks", default="2,8")
ap.add_argument("--variants", default="0,1,2,4,12,13,14,15,16,17,18")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=12)
ap.add_argument("--dtypes", default="f32")
ap.add_argument("--inplace", action="store_true", help="dst = source 0 (the in-place fold of an MPI_IN_PLACE AllReduce)")
ap.add_argument("--shapes", default="", help='nested folds instead of flat variants, e.g. "2,4;4,2;2,2,2": variant 1 '
                                             '= LDS-staged (production), 0 = register kernel (round 1)')
a = ap.parse_args()
lib = ftar.bench_lib()
lib.ftar_debug_reduce_variant.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                                          ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
lib.ftar_debug_reduce_nested_lds.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                                             ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                             ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_void_p]
n = a.elements
shapes = [[int(w) for w in sh.split(",")] for sh in a.shapes.split(";")] if a.shapes else []
if shapes:
    a.ks = ",".join(str(__import__("math").prod(sh)) for sh in shapes)
    a.variants = "0,1"
ks = [int(k) for k in a.ks.split(",")]
setss = [int(x) for x in a.sets.split(",")]
variants = [int(v) for v in a.variants.split(",")]
S = max(setss)
K = max(ks)
bufs = [[torch.rand(n, device="cuda") for _ in range(K + 1)] for _ in range(S)]  # K sources + dst per set
ESZ = {"f32": 4, "bf16": 2, "bf16hop": 2}
# dtype code of ftar_debug_reduce_variant for the ring's bf16 hop fold (rounds after every add; variant 62)
CODE = {"bf16hop": ftar.DTYPE["bf16"] + 100}
stream = torch.cuda.current_stream()
res = {}
for r in range(a.rounds):
    for d in a.dtypes.split(","):
        m = n * 4 // ESZ[d]   # the same bytes per buffer
        for sets in setss:
            for si, k in enumerate(ks):
                arrs = [(ctypes.c_void_p * k)(*[t.data_ptr() for t in bufs[i][:k]]) for i in range(sets)]
                sh = shapes[si] if shapes else None
                sh_c = (ctypes.c_int * len(sh))(*sh) if sh else None
                for v in variants:
                    def launch(i):
                        if sh:
                            return lib.ftar_debug_reduce_nested_lds(v, arrs[i % sets], k, bufs[i % sets][K].data_ptr(),
                                                                    m, ftar.DTYPE[d], sh_c, len(sh), stream.cuda_stream)
                        dst = bufs[i % sets][0 if a.inplace else K].data_ptr()
                        return lib.ftar_debug_reduce_variant(v, CODE.get(d) or ftar.DTYPE[d], arrs[i % sets], k, dst, m,
                                                             stream.cuda_stream)
                    if launch(0) != 0:  # variant not built for this k (or its LDS would exceed 160 KiB)
                        continue
                    for i in range(1, sets):
                        assert launch(i) == 0, (v, k)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    for i in range(a.reps):
                        launch(i)
                    e1.record(stream)
                    torch.cuda.synchronize()
                    key = (d, sets, ",".join(map(str, sh)) if sh else k, v)
                    res.setdefault(key, []).append(e0.elapsed_time(e1) / a.reps)
for (d, sets, k, v), ts in sorted(res.items(), key=lambda kv: str(kv[0])):
    med = statistics.median(ts)
    kk = __import__("math").prod(int(w) for w in str(k).split(","))
    byts = (kk + 1) * n * 4
    print(json.dumps({"dtype": d, "sets": sets, "k": k, "variant": v, "inplace": a.inplace, "bytes_per_buffer": n * 4,
                      "ms_med": round(med, 4),
                      "GBps_med": round(byts / med / 1e6, 1), "GBps_max": round(byts / min(ts) / 1e6, 1)}), flush=True)
