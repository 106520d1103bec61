#!/usr/bin/env python3
"""The host enqueue cost of the N > 1 sweep as a table, from one bench.py line.

    python tools/enqueue_table.py BENCH_JSON [--bound-ms 3.5]

Every sweep entry carries `enqueue_ms`: the median host time one ftar_allreduce call took to return (it
returns once everything is enqueued), max over ranks.  Printed per entry with the pieces per round, the groups
the call enqueued (one per piece per round) and the time per group, next to the call's measured time and to
`--bound-ms`, the 7-link bound of C4's 1 GiB bucket (2 x 7/8 GiB over 7 x 76.8 GB/s = 3.5 ms): an enqueue
above ~10 % of that bound would make the low end of the piece sweep host-bound on an 8-GPU node.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rounds_of(form, topology, world):
    """p2p rounds one call enqueues per piece: direct 2, the reference's stages 2(P-1) (ring) or 2 x stages"""
    base = form.split(":")[0]
    if base in ("direct", "collective"):
        return 2 if base == "direct" else 1
    if base == "stages":
        return 2 * (world - 1) if topology == "ring" else 2 * len(topology.split("+")[0].split(","))
    return None   # peer forms: barriers and whole-block kernels, no pieces


def main():
    import bench
    ap = argparse.ArgumentParser()
    ap.add_argument("line")
    ap.add_argument("--bound-ms", type=float, default=3.5)
    a = ap.parse_args()
    with open(a.line) as f:
        d = json.loads([ln for ln in f if ln.startswith("{")][-1])
    world = d["n_gpus"]
    bucket = d["config"]["bucket_bytes"]
    esz = 2 if d.get("dtype") == "bf16" else 4
    print(f"| topology | form | piece | pieces/round | groups | enqueue ms | us/group | call ms | enqueue / {a.bound_ms} ms |")
    print("|---|---|---|---|---|---|---|---|---|")
    for r in d.get("sweep", []):
        if "ms" not in r or r.get("enqueue_ms") is None:
            continue
        rounds = rounds_of(r["form"], r["topology"], world)
        m = bench.pieces_per_round(r["chunk_bytes"], world, bucket, esz)
        groups = rounds * m if rounds else None
        per = f"{r['enqueue_ms'] * 1e3 / groups:.1f}" if groups else "-"
        piece = f"{r['chunk_bytes'] >> 10} KiB" if r["chunk_bytes"] else "-"
        print(f"| {r['topology']} | {r['form']} | {piece} | {m if rounds else '-'} | {groups or '-'} | "
              f"{r['enqueue_ms']:.3f} | {per} | {r['ms']:.2f} | {r['enqueue_ms'] / a.bound_ms:.2f} |")


if __name__ == "__main__":
    main()
