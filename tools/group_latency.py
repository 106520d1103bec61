#!/usr/bin/env python3
"""Wall time of the in-process group call (ftar_allreduce_group) on one GPU, small buckets to large: P ranks
on cuda:0, tree(P) direct, fp32, from the call to its completion (torch.cuda.synchronize after it), and to the
call's return (it returns once enqueued).  At small buckets this is the host path itself -- the ranks' threads,
the transport's rendezvous, the event plumbing.

    python3 tools/group_latency.py [--ranks 8] [--calls 200]      # FTAR_LIB=<other libftar.so> for an A/B
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "allreduce-over-mpi_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--sizes", default="4096,262144,4194304,67108864")
    a = ap.parse_args()
    import torch
    import ftar
    dev = torch.device("cuda:0")
    g = ftar.Comm.init_local(a.ranks)
    out = {"lib": ftar.LIB_PATH, "ranks": a.ranks, "rows": []}
    try:
        g.set_form("direct")
        for nbytes in (int(x) for x in a.sizes.split(",")):
            n = nbytes // 4
            xs = [torch.full((n,), float(r + 1), device=dev) for r in range(a.ranks)]
            ys = [torch.empty_like(x) for x in xs]
            streams = [torch.cuda.current_stream()] * a.ranks
            calls = a.calls if nbytes <= (4 << 20) else max(10, a.calls // 10)
            for _ in range(5):
                g.allreduce(xs, ys, n, "f32", "sum", topo_=str(a.ranks), streams=streams)
            per, enq = [], []
            torch.cuda.synchronize()
            for _ in range(calls):
                t0 = time.perf_counter()
                g.allreduce(xs, ys, n, "f32", "sum", topo_=str(a.ranks), streams=streams)
                enq.append(time.perf_counter() - t0)
                torch.cuda.synchronize()   # the group call returns once enqueued (since round 5)
                per.append(time.perf_counter() - t0)
            enq.sort()
            want = a.ranks * (a.ranks + 1) / 2
            ok = all(bool((y == want).all()) for y in ys)
            per.sort()
            out["rows"].append({"bytes": nbytes, "calls": calls, "us_median": round(per[len(per) // 2] * 1e6, 1),
                                "us_p10": round(per[len(per) // 10] * 1e6, 1),
                                "us_p90": round(per[9 * len(per) // 10] * 1e6, 1),
                                "us_enqueue_median": round(enq[len(enq) // 2] * 1e6, 1), "check": ok})
            del xs, ys
    finally:
        g.destroy()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
