#!/usr/bin/env python3
"""A/B: bench.py's N = 1 timed loop (K launches of the k = 2 reduce, 4 cold buffer sets in rotation) issued
eagerly on a stream vs the same K launches captured once into a HIP graph and replayed; interleaved rounds,
event-timed on the stream the kernels run on.  Answers whether the inter-launch gaps (ms_per_step minus the
trace's kernel average, ~1 %) shrink when the loop is a graph.

    python tools/graph_loop.py [--rounds 7] [--steps 20]
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "allreduce-over-mpi_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--n", type=int, default=1 << 26)
    a = ap.parse_args()
    import torch

    import ftar
    n, k, sets = a.n, 2, 4
    srcs = [[torch.rand(n, device="cuda") for _ in range(k)] for _ in range(sets)]
    dsts = [torch.empty(n, device="cuda") for _ in range(sets)]
    s = torch.cuda.Stream()
    ptrs = [[t.data_ptr() for t in ss] for ss in srcs]

    def loop():
        for i in range(a.steps):
            ftar.reduce(ptrs[i % sets], dsts[i % sets].data_ptr(), n, "f32", "sum", stream=s)

    with torch.cuda.stream(s):
        loop()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        loop()
    torch.cuda.synchronize()

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        fn()
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.steps

    def replay():
        with torch.cuda.stream(s):
            g.replay()

    res = {"eager": [], "graph": []}
    for _ in range(a.rounds):
        res["eager"].append(timed(loop))
        res["graph"].append(timed(replay))
    gb = (k + 1) * n * 4 / 1e9
    for name, v in res.items():
        med = statistics.median(v)
        print(f"{name:6s} median {med * 1e3:8.2f} us/step = {gb / (med * 1e-3):8.1f} GB/s   all: "
              + " ".join(f"{x * 1e3:.1f}" for x in v))


if __name__ == "__main__":
    main()
