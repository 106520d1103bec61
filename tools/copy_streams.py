#!/usr/bin/env python3
"""PCIe copies from several streams at once, the shape of the host path with 1 or 2 ranks on one GPU
(host_local): each "rank" has an H2D stream and a D2H stream, each moving its own pinned 256 MiB
bucket in 16 MiB pieces (hipMemcpyAsync), all streams at once.  Per case, 10 repetitions: wall time and the
rate per direction.  Cases: 1 or 2 ranks with both directions, 2 ranks with H2D only and D2H only.

    python3 tools/copy_streams.py [--gate]     # --gate: each copy stream first waits on another stream's event
"""
import json
import time

import torch

TOTAL = 256 << 20
N = TOTAL // 4
PIECE = (16 << 20) // 4
dev = torch.device("cuda", 0)


def make(ranks):
    return [{"d": torch.rand(N, device=dev), "hin": torch.rand(N).pin_memory(), "hout": torch.empty(N).pin_memory(),
             "din": torch.empty(N, device=dev), "sh": torch.cuda.Stream(), "sd": torch.cuda.Stream()}
            for _ in range(ranks)]


GATE = {"on": False}   # --gate: every copy stream first waits for an event of another stream (as the host path's do)
gate_stream = torch.cuda.Stream()


def once(rs, h2d, d2h):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if GATE["on"]:
        ev = torch.cuda.Event()
        with torch.cuda.stream(gate_stream):
            torch.cuda._sleep(1)
            ev.record(gate_stream)
        for r in rs:
            r["sh"].wait_event(ev)
            r["sd"].wait_event(ev)
    for i in range(0, N, PIECE):
        for r in rs:
            if h2d:
                with torch.cuda.stream(r["sh"]):
                    r["din"][i:i + PIECE].copy_(r["hin"][i:i + PIECE], non_blocking=True)
            if d2h:
                with torch.cuda.stream(r["sd"]):
                    r["hout"][i:i + PIECE].copy_(r["d"][i:i + PIECE], non_blocking=True)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3


def main():
    import sys
    GATE["on"] = "--gate" in sys.argv
    for ranks, h2d, d2h in [(1, True, True), (2, True, True), (2, True, False), (2, False, True), (1, True, False)]:
        rs = make(ranks)
        once(rs, h2d, d2h)
        ms = [once(rs, h2d, d2h) for _ in range(10)]
        per_dir = ranks * TOTAL / (sorted(ms)[5] * 1e-3) / 1e9
        print(json.dumps({"gate": GATE["on"], "ranks": ranks, "h2d": h2d, "d2h": d2h, "ms_all": [round(m, 2) for m in ms],
                          "ms_median": round(sorted(ms)[5], 2),
                          "GBps_per_direction_median": round(per_dir, 1)}), flush=True)
        del rs


if __name__ == "__main__":
    main()
