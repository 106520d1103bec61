#!/usr/bin/env python3
"""ftar_reduce (the production dispatch) by dtype and k on cold data: launches rotate over 4 disjoint
(k sources + destination) sets of 256 MiB buffers; GB/s of (k+1) x 256 MiB algorithmic bytes, median of
interleaved rounds.  python tools/dtype_rates.py [--ks 2,8] [--dtypes f32,bf16,f64,i32,i16,u8,bool]"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "allreduce-over-mpi_amd"))
import torch  # noqa: E402
import ftar  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ks", default="2,8")
ap.add_argument("--dtypes", default="f32,bf16,f64,i64,i32,i16,u8,bool")
ap.add_argument("--op", default="sum")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=8)
a = ap.parse_args()
NB = 256 << 20
ks = [int(k) for k in a.ks.split(",")]
S = 4
bufs = [[torch.randint(0, 256, (NB,), dtype=torch.uint8, device="cuda") for _ in range(max(ks) + 1)] for _ in range(S)]
stream = torch.cuda.current_stream()
res = {}
for _ in range(a.rounds):
    for d in a.dtypes.split(","):
        n = NB // ftar.dtype_size(d)
        for k in ks:
            def launch(i):
                s = bufs[i % S]
                ftar.reduce(s[:k], s[max(ks)], n, d, a.op, stream=stream)
            for i in range(S):
                launch(i)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i in range(a.reps):
                launch(i)
            e1.record(stream)
            torch.cuda.synchronize()
            res.setdefault((d, k), []).append(e0.elapsed_time(e1) / a.reps)
for (d, k), ts in res.items():
    med = statistics.median(ts)
    print(json.dumps({"dtype": d, "op": a.op, "k": k, "ms_med": round(med, 4),
                      "GBps_med": round((k + 1) * NB / med / 1e6, 1)}), flush=True)
