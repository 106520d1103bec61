#!/usr/bin/env python3
"""Per-launch HBM bytes of the bench kernels from rocprofv3 PMC passes -> profiles/pmc_summary.json.

    python tools/pmc_summary.py FETCH_CSV WRITE_CSV [--elements N] [--k 2,8] [--meta META_JSON] [--source DIR]

One entry per k (bench.py launches the k = 2 headline and the k = 8 line item in the same process); entries
of other workloads already in the summary are kept.  Every entry names the kernel it measured (its template
id, as bench.py's roofline reports the kernel it timed), the sha of the kernel sources and the commit of the
tree the passes ran on (META_JSON, written on the GPU box by tools/gpu_run.sh final): bench.py reports the
traffic only for that kernel built from those sources.

FETCH_SIZE and WRITE_SIZE come from separate `rocprofv3 --pmc` passes (tools/gpu_run.sh pmc).  Per the
gfx950 correction in MI355X_MICROARCH.md: read bytes = 2 x FETCH_SIZE x 1024, write bytes = WRITE_SIZE x 1024.
"""
import argparse
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "allreduce-over-mpi_amd", "ftar"))
from names import kernel_symbol  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("fetch_csv")
ap.add_argument("write_csv")
ap.add_argument("--elements", type=int, default=1 << 26)
ap.add_argument("--k", default="2,8")
ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "pmc_summary.json"))
ap.add_argument("--meta", default="", help="JSON with commit and kernel_sources_sha of the measured tree")
ap.add_argument("--source", default="")
a = ap.parse_args()
meta = {}
if a.meta:
    with open(a.meta) as f:
        meta = json.load(f)


def rows(path, counter, k):
    """the k-way fp32 launches of the bench's own line: the same kernel also runs, on smaller pieces, in the
    line items after it (engine_local's k = 8 folds of 64 MiB pieces, host_local's k = 2 folds of 16 MiB), so
    only launches with the grid of the first one -- the headline (k = 2) or the k8 item (k = 8), which bench.py
    runs before those items -- are kept"""
    with open(path) as f:
        rs = [r for r in csv.DictReader(f) if r["Counter_Name"] == counter and f"F32Sum, {k}," in r["Kernel_Name"]
              and ("reduce_lds_kernel" in r["Kernel_Name"] or "reduce_vec_kernel" in r["Kernel_Name"])]
    return [r for r in rs if r["Grid_Size"] == rs[0]["Grid_Size"]] if rs else rs


def values(path, counter, k):
    return [float(r["Counter_Value"]) for r in rows(path, counter, k)]


try:
    with open(a.out) as f:
        res = json.load(f)
except (OSError, ValueError):
    res = {}
for k in (int(x) for x in a.k.split(",")):
    if not values(a.fetch_csv, "FETCH_SIZE", k):
        continue
    kernels = {kernel_symbol(r["Kernel_Name"]) for r in rows(a.fetch_csv, "FETCH_SIZE", k)}
    kernels_w = {kernel_symbol(r["Kernel_Name"]) for r in rows(a.write_csv, "WRITE_SIZE", k)}
    if len(kernels) != 1 or kernels != kernels_w:
        sys.exit(f"k={k}: the two passes measured different kernels: {kernels} / {kernels_w}")
    fetch = statistics.median(values(a.fetch_csv, "FETCH_SIZE", k))
    write = statistics.median(values(a.write_csv, "WRITE_SIZE", k))
    rd, wr = 2 * fetch * 1024, write * 1024
    key = f"reduce_k{k}_f32_n{a.elements}"
    res[key] = {
        "kernel": kernels.pop(),
        "commit": meta.get("commit"),
        "kernel_sources_sha": meta.get("kernel_sources_sha"),
        "launches": len(values(a.fetch_csv, "FETCH_SIZE", k)),
        "FETCH_SIZE_kB_median": fetch, "WRITE_SIZE_kB_median": write,
        "read_bytes_corrected": rd, "write_bytes": wr, "hbm_bytes_per_launch": rd + wr,
        "algorithmic_bytes_per_launch": (k + 1) * a.elements * 4,
        "traffic_over_algorithmic": round((rd + wr) / ((k + 1) * a.elements * 4), 6),
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (tools/gpu_run.sh pmc); "
                  "read bytes = 2 x FETCH_SIZE x 1024 per the gfx950 correction, write bytes = WRITE_SIZE x 1024",
        "source": a.source or f"{a.fetch_csv}, {a.write_csv}"}
    print(json.dumps({key: res[key]}))
with open(a.out, "w") as f:
    json.dump(res, f, indent=1)
