#!/usr/bin/env python3
"""The engine's two-stream pipeline on one GPU, from a rocprofv3 trace of bench.py's engine_local item.

    rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d OUT -o el -- \\
        python3 bench.py --engine-local-only --steps 5 --warmup 2
    python3 tools/engine_local_trace.py OUT/.../el_kernel_trace.csv [OUT/.../el_memory_copy_trace.csv] \\
        --calls 7 --keep 5 --hbm-bytes <engine_local.hbm_bytes_per_call>

Keeps the engine's own work (ftar's copies and folds, and the runtime's copy kernels and SDMA copies the
in-process transport issues), splits it into the calls at the marker kernels bench.py launches before each
call (torch.cuda._sleep, a "spin" kernel; without markers: consecutive runs of len/calls ops in start
order), keeps the last `keep`, and reports per call:
  * span, device-busy time (union of every kernel and copy), idle = span - busy;
  * the folds (reduce kernels) and the transfers (device copies: blit kernels or SDMA copies): their busy
    time, and how much of the fold time runs while a transfer is in flight;
  * per stream (Stream_Id: the 8 ranks' comm and reduce streams), ops, busy time and the gaps between
    consecutive ops -- the idle time per piece the verdict asks to name;
  * the HBM rate of the call (--hbm-bytes over the span) and over the busy time.
"""
import argparse
import csv
import json
import statistics


def load(path, kind):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("Direction") or r.get("Operation") or kind
            out.append({"kind": kind, "name": name, "stream": r.get("Stream_Id", r.get("Queue_Id", "?")),
                        "s": int(r["Start_Timestamp"]), "e": int(r["End_Timestamp"])})
    return out


def union(iv):
    res = []
    for s, e in sorted(iv):
        if res and s <= res[-1][1]:
            res[-1][1] = max(res[-1][1], e)
        else:
            res.append([s, e])
    return res


def length(u):
    return sum(e - s for s, e in u)


def intersect(a, b):
    """total length of the intersection of two unions"""
    tot, j = 0, 0
    for s, e in a:
        while j < len(b) and b[j][1] <= s:
            j += 1
        k = j
        while k < len(b) and b[k][0] < e:
            tot += max(0, min(e, b[k][1]) - max(s, b[k][0]))
            k += 1
    return tot


def is_fold(name):
    """a reduce kernel of k >= 2 sources; the k = 1 instance (kernarg Srcs<1>) is launch_copy, a transfer"""
    return ("reduce_lds_kernel" in name or "reduce_vec_kernel" in name or "reduce_tree" in name) and \
        "Srcs<1>" not in name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernel_csv")
    ap.add_argument("copy_csv", nargs="?")
    ap.add_argument("--calls", type=int, default=7)
    ap.add_argument("--keep", type=int, default=5)
    ap.add_argument("--hbm-bytes", type=float, default=0.0)
    ap.add_argument("--first", action="store_true",
                    help="the calls follow the FIRST `calls` markers (engine_local's default configuration, before "
                         "its whole-block and peer-read sub-runs add markers of their own), not the last")
    a = ap.parse_args()
    # the engine's own work only: ftar's kernels (folds, copies) and the runtime's copies (the input setup
    # and the sample check around the timed calls are torch kernels)
    kern = load(a.kernel_csv, "kernel")
    marks = sorted(o["s"] for o in kern if "sleep" in o["name"].lower() or "spin" in o["name"].lower())
    mark_end = {o["s"]: o["e"] for o in kern if "sleep" in o["name"].lower() or "spin" in o["name"].lower()}
    ops = [o for o in kern if "ftar::" in o["name"] or "copyBuffer" in o["name"]]
    if a.copy_csv:
        ops += load(a.copy_csv, "copy")
    ops.sort(key=lambda o: o["s"])
    if len(marks) >= a.calls:   # the calls lie between consecutive markers (the last one: up to the next torch op)
        if a.first:
            bounds = marks[:a.calls] + [marks[a.calls] if len(marks) > a.calls else max(o["e"] for o in ops) + 1]
        else:
            bounds = marks[-a.calls:] + [max(o["e"] for o in ops) + 1]
        calls = [[o for o in ops if lo <= o["s"] < hi] for lo, hi in zip(bounds, bounds[1:])]
        # the last call ends where its ops stop: drop anything after a gap wider than the call itself
        last = calls[-1]
        for i in range(1, len(last)):
            if last[i]["s"] - max(x["e"] for x in last[:i]) > 1e6:   # 1 ms of silence: the sample check
                calls[-1] = last[:i]
                break
    else:
        if len(ops) % a.calls:
            raise SystemExit(f"{len(ops)} engine ops do not split into {a.calls} equal calls")
        per = len(ops) // a.calls
        calls = [ops[i * per:(i + 1) * per] for i in range(a.calls)]
    res = []
    starts = bounds[:-1] if len(marks) >= a.calls else [None] * len(calls)
    for c, mk in list(zip(calls, starts))[-a.keep:]:
        span = (min(o["s"] for o in c), max(o["e"] for o in c))
        busy = union([(o["s"], o["e"]) for o in c])
        folds = union([(o["s"], o["e"]) for o in c if is_fold(o["name"])])
        xfer = union([(o["s"], o["e"]) for o in c if not is_fold(o["name"])])
        streams = {}
        for o in c:
            streams.setdefault(o["stream"], []).append(o)
        per_stream = []
        for sid, so in sorted(streams.items(), key=lambda kv: kv[1][0]["s"]):
            so.sort(key=lambda o: o["s"])
            g = [max(0, so[i]["s"] - so[i - 1]["e"]) for i in range(1, len(so))]
            per_stream.append({"stream": sid, "ops": len(so), "folds": sum(is_fold(o["name"]) for o in so),
                               "busy_us": round(length(union([(o["s"], o["e"]) for o in so])) / 1e3, 1),
                               "first_us": round((so[0]["s"] - span[0]) / 1e3, 1),
                               "last_end_us": round((so[-1]["e"] - span[0]) / 1e3, 1),
                               "gaps_us": [round(x / 1e3, 1) for x in g]})
        fold_t = length(folds)
        d = {"span_us": round((span[1] - span[0]) / 1e3, 1), "busy_us": round(length(busy) / 1e3, 1),
             "idle_us": round((span[1] - span[0] - length(busy)) / 1e3, 1),
             "fold_busy_us": round(fold_t / 1e3, 1), "transfer_busy_us": round(length(xfer) / 1e3, 1),
             "fold_overlapped_by_transfers": round(intersect(folds, xfer) / fold_t, 4) if fold_t else None,
             "ops": len(c), "fold_ops": sum(is_fold(o["name"]) for o in c),
             "kernel_time_sum_over_span": round(sum(o["e"] - o["s"] for o in c) / (span[1] - span[0]), 2),
             "streams": per_stream}
        if mk is not None:   # from the marker kernel's end (the call's start on the host) to its first kernel
            d["lead_us"] = round((span[0] - mark_end[mk]) / 1e3, 1)
        if a.hbm_bytes:
            d["hbm_GBps_over_span"] = round(a.hbm_bytes / (span[1] - span[0]), 1)
            d["hbm_GBps_over_busy"] = round(a.hbm_bytes / length(busy), 1)
        res.append(d)
    names = {}
    for o in ops:
        names.setdefault(o["name"][:90], []).append(o["e"] - o["s"])
    summary = {"calls_found": len(calls), "kept": len(res), "markers": len(marks),
               "median_span_us": statistics.median(r["span_us"] for r in res),
               "median_idle_us": statistics.median(r["idle_us"] for r in res),
               "median_fold_overlap": statistics.median(r["fold_overlapped_by_transfers"] or 0 for r in res),
               "median_lead_us": statistics.median(r["lead_us"] for r in res) if "lead_us" in res[0] else None,
               "op_kinds": {k: {"count": len(v), "mean_us": round(statistics.mean(v) / 1e3, 1)}
                            for k, v in sorted(names.items(), key=lambda kv: -sum(kv[1]))[:8]},
               "calls": res}
    if a.hbm_bytes:
        summary["median_hbm_GBps_over_span"] = statistics.median(r["hbm_GBps_over_span"] for r in res)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
