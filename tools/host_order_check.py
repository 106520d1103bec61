#!/usr/bin/env python3
"""Happens-before check of one peer_allreduce_host call (the MPI drop-in's `ipc` host path) from a rocprofv3
kernel + memory-copy trace of every rank: every read of a piece range must start after its writer ended.

    bash tools/gpu_run.sh hbtrace          # 8 processes, one c4_host_read call, FTAR_STRESS_PIDMAP
    python3 tools/host_order_check.py gpurun_out/hbtrace --pidmap gpurun_out/pidmap.txt --topo ring

The call, per rank r and piece k (engine_host.cpp; piece k = elements [k*c, (k+1)*c) of every block, blocks
in order, one copy each):
  H2D(r,k)    P SDMA copies on r's H2D stream: r's input, piece k of every block, into r's X
  fold(r,k)   the reduce kernel on r's comm stream: reads piece k of block o(r) from every rank's X (over the
              IPC mapping), writes it into r's X (ring: o(r) = r + 1 mod P, tree(P): o(r) = r)
  gather(r,k) the gather kernel on r's comm stream: copies piece k of every other block from its owner's X
              into r's X
  D2H(r,k)    P copies (blit kernels or SDMA) on r's D2H stream: piece k of every block of r's X -> host
Edges (reader start - writer end = slack; a negative slack is a violation):
  h2d->fold        H2D(r,k)[o(q)] -> fold(q,k) for every r, q     (fold reads r's input)
  fold->gather     fold(q,k) -> gather(r,k) for every q != r       (gather reads q's final piece; also: r's
                                                                    gather overwrites what q's fold read)
  gather->d2h      gather(r,k) -> D2H(r,k)[b] for every b != o(r)  (D2H reads what the gather wrote)
  fold->d2h        fold(r,k) -> D2H(r,k)[o(r)]                     (D2H of r's own block)
  d2h->next_h2d    none: a later piece's H2D never touches piece k
Prints a JSON summary (per edge: count, min slack in us, violations) and exits 1 on any violation.

    python3 tools/host_order_check.py --marks gpurun_out/stress.jsonl

checks the local edges of every rank-call from the engine's own hand-off marks instead (phase timing, recorded
by tools/host_comm_stress.py under FTAR_STRESS_MARKS=1), with no profiler.
"""
import argparse
import csv
import glob
import json
import os
import re
import sys


def load_dir(d):
    """{pid: {"k": [kernel rows], "m": [memory copy rows]}} from a rocprofv3 -d directory."""
    out = {}
    for path in glob.glob(os.path.join(d, "**", "*_kernel_trace.csv"), recursive=True) + \
            glob.glob(os.path.join(d, "**", "*_memory_copy_trace.csv"), recursive=True):
        m = re.search(r"(\d+)_(kernel|memory_copy)_trace\.csv$", os.path.basename(path))
        if not m:
            continue
        pid, kind = int(m.group(1)), m.group(2)
        rows = []
        with open(path) as f:
            for r in csv.DictReader(f):
                rows.append({"name": r.get("Kernel_Name") or r.get("Direction", ""), "stream": r.get("Stream_Id"),
                             "s": int(r["Start_Timestamp"]), "e": int(r["End_Timestamp"])})
        out.setdefault(pid, {"k": [], "m": []})["k" if kind == "kernel" else "m"].extend(rows)
    return out


def ops_of_rank(t, P):
    """The call's operations of one rank, in issue order: fold[k], gather[k], h2d[k][b], d2h[k][b]."""
    ks = sorted(t["k"], key=lambda r: r["s"])
    gathers = [r for r in ks if "gather_kernel" in r["name"]]
    if not gathers:
        raise ValueError("no gather kernels in this trace")
    comm = gathers[0]["stream"]
    on_comm = [r for r in ks if r["stream"] == comm]
    folds = [r for r in on_comm if "reduce" in r["name"]]
    gathers = [r for r in on_comm if "gather_kernel" in r["name"]]
    m = len(gathers)
    if len(folds) != m:
        raise ValueError(f"{len(folds)} folds vs {m} gathers on the comm stream")
    by_stream = {}
    for r in t["m"]:
        if r["name"].endswith("HOST_TO_DEVICE"):
            by_stream.setdefault(("h2d", r["stream"]), []).append(r)
        elif r["name"].endswith("DEVICE_TO_HOST"):
            by_stream.setdefault(("d2h", r["stream"]), []).append(r)
    for r in ks:   # D2H as the runtime's blit kernels
        if "copyBuffer" in r["name"] and r["stream"] != comm:
            by_stream.setdefault(("blit", r["stream"]), []).append(r)
    want = m * P
    h2d = [v for (kind, _), v in by_stream.items() if kind == "h2d" and len(v) >= want]
    d2h = [v for (kind, _), v in by_stream.items() if kind in ("d2h", "blit") and len(v) >= want]
    if not h2d or not d2h:
        raise ValueError(f"no stream with {want} H2D / D2H copies: "
                         f"{ {k: len(v) for k, v in by_stream.items()} }")
    # the traced run makes this one call: its copies are the first `want` on their streams
    h2d = sorted(max(h2d, key=len), key=lambda r: r["s"])[:want]
    d2h = sorted(max(d2h, key=len), key=lambda r: r["s"])[:want]
    return {"fold": folds, "gather": gathers, "h2d": [h2d[k * P:(k + 1) * P] for k in range(m)],
            "d2h": [d2h[k * P:(k + 1) * P] for k in range(m)], "m": m}


def check(ranks, topo):
    P = len(ranks)
    own = (lambda r: (r + 1) % P) if topo == "ring" else (lambda r: r)
    m = ranks[0]["m"]
    edges = {}

    def edge(name, w, rd, what):
        sl = (rd["s"] - w["e"]) / 1e3
        e = edges.setdefault(name, {"count": 0, "min_slack_us": None, "violations": []})
        e["count"] += 1
        e["min_slack_us"] = sl if e["min_slack_us"] is None else min(e["min_slack_us"], sl)
        if sl < 0:
            e["violations"].append(dict(what, slack_us=round(sl, 3)))

    for k in range(m):
        for q in range(P):
            for r in range(P):
                edge("h2d->fold", ranks[r]["h2d"][k][own(q)], ranks[q]["fold"][k], {"piece": k, "h2d_rank": r, "fold_rank": q})
                if q != r:
                    edge("fold->gather", ranks[q]["fold"][k], ranks[r]["gather"][k], {"piece": k, "fold_rank": q, "gather_rank": r})
        for r in range(P):
            for b in range(P):
                if b == own(r):
                    edge("fold->d2h", ranks[r]["fold"][k], ranks[r]["d2h"][k][b], {"piece": k, "rank": r, "block": b})
                else:
                    edge("gather->d2h", ranks[r]["gather"][k], ranks[r]["d2h"][k][b], {"piece": k, "rank": r, "block": b})
    for e in edges.values():
        e["min_slack_us"] = round(e["min_slack_us"], 3)
        e["nviolations"] = len(e["violations"])
        e["violations"] = e["violations"][:10]
    return edges


def check_marks(phases):
    """The same edges inside one rank from the engine's own hand-off marks (phase timing: each mark is the time its
    stream reached it, in ms since the call's start on the same device): H2D(k) done before my fold(k) starts, my
    fold(k) done before my gather(k) starts, my gather(k) done before my D2H(k) starts, every D2H done before the
    call's last barrier.  The cross-process edges are host barriers and need no clock."""
    t = {}
    for name, ms in phases:
        t[name] = ms
    ks = sorted(int(n.split()[1]) for n in t if n.startswith("gather ") and n.endswith(" done"))
    edges = {}

    def edge(name, w, r, k):
        if w not in t or r not in t:
            return
        sl = (t[r] - t[w]) * 1e3   # us
        e = edges.setdefault(name, {"count": 0, "min_slack_us": None, "violations": []})
        e["count"] += 1
        e["min_slack_us"] = sl if e["min_slack_us"] is None else min(e["min_slack_us"], sl)
        if sl < 0:
            e["violations"].append({"piece": k, "slack_us": round(sl, 3)})
    for k in ks:
        edge("h2d->fold", f"h2d {k} done", f"fold {k} start", k)
        edge("fold->gather", f"fold {k} done", f"gather {k} start", k)
        edge("gather->d2h", f"gather {k} done", f"d2h {k} start", k)
        edge("d2h->last barrier", f"d2h {k} done", "barrier", k)
    for e in edges.values():
        e["min_slack_us"] = round(e["min_slack_us"], 3)
        e["nviolations"] = len(e["violations"])
    return {"pieces": len(ks), "edges": edges, "ok": bool(ks) and all(e["nviolations"] == 0 for e in edges.values())}


def main_marks(path, out):
    """every rank-call of a host_comm_stress.py --out file run with FTAR_STRESS_MARKS=1"""
    res = {"calls": 0, "ok": True, "edges": {}}
    with open(path) as f:
        for ln in f:
            d = json.loads(ln)
            if not d.get("phases"):
                continue
            c = check_marks(d["phases"])
            res["calls"] += 1
            res["ok"] = res["ok"] and c["ok"]
            for name, e in c["edges"].items():
                a = res["edges"].setdefault(name, {"count": 0, "min_slack_us": None, "nviolations": 0})
                a["count"] += e["count"]
                a["nviolations"] += e["nviolations"]
                a["min_slack_us"] = e["min_slack_us"] if a["min_slack_us"] is None else min(a["min_slack_us"], e["min_slack_us"])
    res["ok"] = res["ok"] and res["calls"] > 0
    s = json.dumps(res, indent=1)
    print(s)
    if out:
        with open(out, "w") as f:
            f.write(s + "\n")
    return 0 if res["ok"] else 1


def main():
    if "--marks" in sys.argv:   # host_order_check.py --marks stress.jsonl [--out f]
        i = sys.argv.index("--marks")
        out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else ""
        return main_marks(sys.argv[i + 1], out)
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--pidmap", required=True, help="lines 'rank pid' (FTAR_STRESS_PIDMAP)")
    ap.add_argument("--topo", choices=["ring", "tree"], default="ring")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    pid_rank = {}
    with open(a.pidmap) as f:
        for ln in f:
            r, p = ln.split()
            pid_rank[int(p)] = int(r)
    traces = load_dir(a.trace_dir)
    P = len(pid_rank)
    ranks = [None] * P
    for pid, t in traces.items():
        if pid in pid_rank:
            ranks[pid_rank[pid]] = ops_of_rank(t, P)
    missing = [r for r in range(P) if ranks[r] is None]
    if missing:
        raise SystemExit(f"no trace for ranks {missing} (pids {sorted(traces)})")
    edges = check(ranks, a.topo)
    t0 = min(r["h2d"][0][0]["s"] for r in ranks)
    res = {"ranks": P, "pieces": ranks[0]["m"], "edges": edges,
           "call_span_ms": round((max(r["d2h"][-1][-1]["e"] for r in ranks) - t0) / 1e6, 3),
           "ok": all(e["nviolations"] == 0 for e in edges.values())}
    s = json.dumps(res, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")
    return 0 if res["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
