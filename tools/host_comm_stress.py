#!/usr/bin/env python3
"""Diagnostic: the full-size host-comm cases (tests/host_comm_cases.py) for many cycles on eight processes of
one GPU, each case on poisoned exchange buffers, every mapping compared page by page, every wrong result
localised and classified -- under the current settings and under round 5's failing configuration.

    python3 tools/host_comm_stress.py --config current --cycles 10 --out gpurun_out/stress.jsonl
    python3 tools/host_comm_stress.py --config r5 --cycles 10 ...

Configurations (environment of every rank; engine.cpp ensure_host_streams, engine_host.cpp): see CONFIGS.
  current  the tree as it is
  r5       the build of round 5's one c4_host_read mismatch: copy streams at the highest priority
           (FTAR_DEBUG_HOST_COPY_PRIORITY=1), every H2D piece issued up front (FTAR_DEBUG_HOST_LOOKAHEAD=1000),
           D2H on the host D2H stream (FTAR_DEBUG_HOST_D2H_STREAM=1); prio / upfront / d2hs one of those each
  r5_*     r5 with a change at the gather -> D2H hand-off (FTAR_DEBUG_HOST_GATHER_FENCE): an empty kernel
           after the gather (noop), a system-scope release ending every gather workgroup (fence), temporal
           stores in the gather (temporal); r5_log / log: a record per gather workgroup (gather_forensics)
Writes one JSON line per (rank, cycle, case) and prints a summary; exit status 1 if anything was wrong.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "allreduce-over-mpi_amd"), os.path.join(ROOT, "tests")]

R5 = {"FTAR_DEBUG_HOST_COPY_PRIORITY": "1", "FTAR_DEBUG_HOST_LOOKAHEAD": "1000", "FTAR_DEBUG_HOST_D2H_STREAM": "1"}
CONFIGS = {
    "current": {},
    "r5": R5,
    # one ingredient of r5 at a time
    "prio": {"FTAR_DEBUG_HOST_COPY_PRIORITY": "1"},
    "upfront": {"FTAR_DEBUG_HOST_LOOKAHEAD": "1000"},
    "d2hs": {"FTAR_DEBUG_HOST_D2H_STREAM": "1"},
    # r5 with a change at the gather -> D2H hand-off (FTAR_DEBUG_HOST_GATHER_FENCE, engine_host.cpp)
    "r5_noop": dict(R5, FTAR_DEBUG_HOST_GATHER_FENCE="1"),
    "r5_fence": dict(R5, FTAR_DEBUG_HOST_GATHER_FENCE="2"),
    "r5_temporal": dict(R5, FTAR_DEBUG_HOST_GATHER_FENCE="3"),
    "fence": {"FTAR_DEBUG_HOST_GATHER_FENCE": "2"},
    # pairs of r5's ingredients, and r5 with the D2H ordered by the host instead of an event
    "prio_d2hs": {"FTAR_DEBUG_HOST_COPY_PRIORITY": "1", "FTAR_DEBUG_HOST_D2H_STREAM": "1"},
    "prio_upfront": {"FTAR_DEBUG_HOST_COPY_PRIORITY": "1", "FTAR_DEBUG_HOST_LOOKAHEAD": "1000"},
    "r5_hostorder": dict(R5, FTAR_DEBUG_HOST_D2H_ORDER="host"),
    # a record per gather workgroup (FTAR_DEBUG_HOST_GATHER_LOG): where and when each ran, and whether its
    # last store reached host memory (past the caches) and device memory (through them)
    "log": {"FTAR_DEBUG_HOST_GATHER_LOG": "1"},
    "r5_log": dict(R5, FTAR_DEBUG_HOST_GATHER_LOG="1"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=sorted(CONFIGS), default="current")
    ap.add_argument("--cycles", type=int, default=5)
    ap.add_argument("--cases", default="", help="comma-separated case names (default: the four default cases)")
    ap.add_argument("--out", default="")
    ap.add_argument("--timeout", type=int, default=600)
    ap.add_argument("--world", type=int, default=8, help="processes (ranks) on the one GPU, 2..8")
    a = ap.parse_args()
    import host_comm_cases as hc
    cases = hc.CASES + hc.WIDE
    if a.cases:
        want = a.cases.split(",")
        cases = [c for c in cases if c[0] in want]
    t0 = time.time()
    if not 2 <= a.world <= 8:
        sys.exit("--world must be 2..8")
    res = hc.run(cases, world=a.world, cycles=a.cycles, env=CONFIGS[a.config], timeout=a.timeout)
    lines = hc.failures(res, world=a.world)
    if a.out:
        with open(a.out, "a") as f:
            for r in sorted(res):
                for x in res[r].get("results", []):
                    f.write(json.dumps(dict(x, rank=r, config=a.config, world=a.world)) + "\n")
                if "error" in res[r]:
                    f.write(json.dumps({"rank": r, "config": a.config, "error": res[r]["error"]}) + "\n")
    ms = {}
    for r in res:
        for x in res[r].get("results", []):
            ms.setdefault(x["name"], []).append(x["ms"])
    glog = {}
    for r in res:
        for x in res[r].get("results", []):
            for key, v in x.get("gather_log", {}).items():
                if key in ("wgs", "host_missing", "dev_missing", "runs", "ids_run_twice", "xcc_is_w_mod_8",
                           "split_pieces"):
                    glog[key] = glog.get(key, 0) + v
                elif key == "queues":
                    for q, c in v.items():
                        glog.setdefault("queues", {})[q] = glog.get("queues", {}).get(q, 0) + c
    print(json.dumps({"config": a.config, "world": a.world, "cycles": a.cycles, "cases": [c[0] for c in cases],
                      "problems": len(lines), "seconds": round(time.time() - t0, 1),
                      "median_ms": {k: sorted(v)[len(v) // 2] for k, v in ms.items()},
                      **({"gather_log": glog} if glog else {})}))
    for ln in lines:
        print(ln)
    return 1 if lines else 0


if __name__ == "__main__":
    sys.exit(main())
