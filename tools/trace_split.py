#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace of `python bench.py` (N = 1) into the bench's launch phases.

    python tools/trace_split.py run_kernel_trace.csv [--steps 20 --warmup 5 --sets 4] [--out summary.json]

rocprofv3 --stats averages every dispatch of a kernel symbol, and bench.py launches the headline kernel in two
regimes (buffer sets in rotation -- the headline -- and the reference harness's same-buffer loop) plus a
spot check, so the stats average mixes them.  bench.py's launch order is fixed (bench_single):

    k = 2:  W rotating warmup, K rotating timed, W same-buffer warmup, K same-buffer timed, `sets` spot-check
    k = 8:  2 untimed, 20 timed out of place, 20 timed in place

This tool takes the dispatches of each kernel in start order and averages each phase, so the headline's
kernel duration can be compared with the bench line's per-step time."""
import argparse
import csv
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "allreduce-over-mpi_amd",
                                "ftar"))
from names import kernel_symbol  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--sets", type=int, default=4)
ap.add_argument("--k8-reps", type=int, default=20)
ap.add_argument("--out", default="")
a = ap.parse_args()

rows = []
with open(a.trace) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kernel_symbol(r["Kernel_Name"])))
rows.sort()


def phases(sym, spec):
    d = [(e - s) / 1e3 for s, e, k in rows if k == sym]
    out, i = {}, 0
    for name, cnt in spec:
        seg = d[i:i + cnt]
        i += cnt
        if name and seg:
            out[name] = {"launches": len(seg), "avg_us": round(statistics.mean(seg), 3),
                         "median_us": round(statistics.median(seg), 3), "min_us": round(min(seg), 3),
                         "max_us": round(max(seg), 3)}
    out["dispatches_total"] = len(d)
    return out


syms = sorted({k for _, _, k in rows if k.startswith("reduce_lds_kernel<F32Sum")})
res = {"trace": os.path.relpath(a.trace), "kernels": {}}
for sym in syms:
    kk = int(sym.split(",")[1])
    if kk == 2:
        spec = [(None, a.warmup), ("rotating_timed", a.steps), (None, a.warmup), ("same_buffers_timed", a.steps),
                ("spot_check", a.sets)]
        algo = 3 * (1 << 26) * 4
    else:
        spec = [(None, 2), ("out_of_place_timed", a.k8_reps), ("in_place_timed", a.k8_reps)]
        algo = (kk + 1) * (1 << 26) * 4
    ph = phases(sym, spec)
    for name, v in ph.items():
        if isinstance(v, dict):
            v["GBps_at_avg"] = round(algo / (v["avg_us"] * 1e-6) / 1e9, 1)
    res["kernels"][sym] = ph
print(json.dumps(res, indent=1))
if a.out:
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
