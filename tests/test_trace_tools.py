"""The trace analyser behind DESIGN §9's engine_local numbers (tools/engine_local_trace.py), on a small synthetic
rocprofv3 kernel trace whose answers are known: calls split at the marker kernels, span / busy / idle, fold
time overlapped by transfers, per-stream gaps, the lead from a marker's end to the call's first kernel, and
the HBM rate over the span."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "tools", "engine_local_trace.py")

FOLD = "void ftar::(anonymous namespace)::reduce_lds_kernel<ftar::(anonymous namespace)::F32Sum, 8>(Srcs<8>)"
COPY = "void ftar::(anonymous namespace)::reduce_lds_kernel<ftar::(anonymous namespace)::SwarSum<u>(Srcs<1>)"
MARK = "void at::native::sleep_kernel(long)"


def write_trace(path):
    """Two calls.  Each: a marker ending 10 us before the call's first op; a copy on stream 1 (0-100 us after
    the call start), a fold on stream 2 (50-150 us: half of it under the copy), a second copy on stream 1
    (200-300 us: 50 us of idle device before it).  Times in ns."""
    rows = []

    def add(name, sid, s, e):
        rows.append({"Kernel_Name": name, "Stream_Id": sid, "Start_Timestamp": s, "End_Timestamp": e})
    for base in (1_000_000, 2_000_000):
        add(MARK, 0, base - 20_000, base - 10_000)
        add(COPY, 1, base, base + 100_000)
        add(FOLD, 2, base + 50_000, base + 150_000)
        add(COPY, 1, base + 200_000, base + 300_000)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)


def test_engine_local_trace_on_a_known_trace(tmp_path):
    p = tmp_path / "k.csv"
    write_trace(p)
    out = subprocess.run([sys.executable, TOOL, str(p), "--calls", "2", "--keep", "2", "--hbm-bytes", "300000"],
                         capture_output=True, text=True, check=True).stdout
    d = json.loads(out)
    assert d["calls_found"] == 2 and d["kept"] == 2 and d["markers"] == 2
    for c in d["calls"]:
        assert c["span_us"] == 300.0 and c["busy_us"] == 250.0 and c["idle_us"] == 50.0
        assert c["fold_busy_us"] == 100.0 and c["transfer_busy_us"] == 200.0
        assert c["fold_overlapped_by_transfers"] == 0.5        # 50 of the fold's 100 us under the first copy
        assert c["ops"] == 3 and c["fold_ops"] == 1 and c["lead_us"] == 10.0
        assert c["hbm_GBps_over_span"] == 1.0                   # 300,000 B over 300 us
        by = {s["stream"]: s for s in c["streams"]}
        assert by["1"]["gaps_us"] == [100.0] and by["2"]["folds"] == 1
    assert d["median_idle_us"] == 50.0 and d["median_fold_overlap"] == 0.5


def test_scale_report_on_the_rehearsed_n8_line():
    """tools/scale_report.py, which reads the driver's N > 1 lines, on the P = 8 line rehearsed over RCCL
    loopback on round 5's final tree (profiles/r05/loopback_final/dist8.json): every section it prints."""
    line = os.path.join(ROOT, "profiles", "r05", "loopback_final", "dist8.json")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "scale_report.py"), line],
                         capture_output=True, text=True, check=True).stdout
    for needle in ("== N=8:", "rccl_p2p_best:", "c4_ring direct (gather + ring-order fold)", "<- judged",
                   "xGMI probe", "cost model refit", "unidentified", "C5 bf16:", "a tie of 6 broken by stages",
                   "host e2e:", "bit-identical to the device path", "stages (s):"):
        assert needle in out, (needle, out[:3000])


HOST_ORDER = os.path.join(ROOT, "tools", "host_order_check.py")
GATHER = "void ftar::(anonymous namespace)::gather_kernel(ftar::(anonymous namespace)::SegArgs, int)"
BLIT = "__amd_rocclr_copyBuffer"


def write_host_call(d, P=4, m=3, late=None):
    """A well-ordered peer_allreduce_host call of P ranks and m pieces, one rocprofv3 kernel + memory-copy
    trace per pid (100 + rank), in us steps: piece k's H2D copies at [10k, 10k+5), every fold at
    [100k+20, 100k+30), every gather at [100k+40, 100k+50), the D2H blits at [100k+60, 100k+65).  late =
    (rank, piece): that rank's D2H of that piece starts before its gather ends (the violation to find)."""
    os.makedirs(d, exist_ok=True)
    us = 1000
    with open(os.path.join(d, "pidmap.txt"), "w") as f:
        for r in range(P):
            f.write(f"{r} {100 + r}\n")
    for r in range(P):
        ks, ms = [], []
        for k in range(m):
            t = 100 * k
            ks.append({"Kernel_Name": FOLD, "Stream_Id": 1, "Start_Timestamp": (t + 20) * us, "End_Timestamp": (t + 30) * us})
            ks.append({"Kernel_Name": GATHER, "Stream_Id": 1, "Start_Timestamp": (t + 40) * us, "End_Timestamp": (t + 50) * us})
            d2h0 = t + (45 if late == (r, k) else 60)
            for b in range(P):
                ms.append({"Direction": "MEMORY_COPY_HOST_TO_DEVICE", "Stream_Id": 3,
                           "Start_Timestamp": (10 * k) * us + b, "End_Timestamp": (10 * k + 5) * us + b})
                ks.append({"Kernel_Name": BLIT, "Stream_Id": 2, "Start_Timestamp": d2h0 * us + b,
                           "End_Timestamp": (d2h0 + 5) * us + b})
        for rows, kind in ((ks, "kernel"), (ms, "memory_copy")):
            with open(os.path.join(d, f"{100 + r}_{kind}_trace.csv"), "w", newline="") as f:
                w = csv.DictWriter(f, fieldnames=list(rows[0]))
                w.writeheader()
                w.writerows(rows)


def test_host_order_check_on_known_calls(tmp_path):
    good = tmp_path / "good"
    write_host_call(str(good))
    r = subprocess.run([sys.executable, HOST_ORDER, str(good), "--pidmap", str(good / "pidmap.txt")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout)
    assert d["ok"] and d["ranks"] == 4 and d["pieces"] == 3
    e = d["edges"]
    assert e["h2d->fold"]["count"] == 3 * 4 * 4 and e["fold->gather"]["count"] == 3 * 4 * 3
    assert e["gather->d2h"]["count"] == 3 * 4 * 3 and e["fold->d2h"]["count"] == 3 * 4
    assert e["fold->gather"]["min_slack_us"] == 10.0 and e["gather->d2h"]["min_slack_us"] == 10.0
    bad = tmp_path / "bad"
    write_host_call(str(bad), late=(1, 2))
    r = subprocess.run([sys.executable, HOST_ORDER, str(bad), "--pidmap", str(bad / "pidmap.txt")],
                       capture_output=True, text=True)
    assert r.returncode == 1
    v = json.loads(r.stdout)["edges"]["gather->d2h"]
    assert v["nviolations"] == 3 and {x["rank"] for x in v["violations"]} == {1} and {x["piece"] for x in v["violations"]} == {2}


def test_host_order_check_from_the_engines_marks(tmp_path):
    """--marks: the local hand-off edges of peer_allreduce_host from its phase-timing marks (ms since the call's
    start), one JSON line per rank-call as tools/host_comm_stress.py writes them; one late D2H is found."""
    def phases(late=None):
        ph = [["start", 0.0]]
        for k in range(3):
            t = 10.0 * k
            ph += [[f"h2d {k} done", t + 1], [f"fold {k} start", t + 2], [f"fold {k} done", t + 3],
                   [f"gather {k} start", t + 4], [f"gather {k} done", t + 5],
                   [f"d2h {k} start", t + (4.5 if late == k else 6)], [f"d2h {k} done", t + 7]]
        return ph + [["barrier", 40.0]]
    good = tmp_path / "good.jsonl"
    good.write_text("\n".join(json.dumps({"rank": r, "name": "c4_host_read", "phases": phases()}) for r in range(4)) + "\n")
    r = subprocess.run([sys.executable, HOST_ORDER, "--marks", str(good)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    d = json.loads(r.stdout)
    assert d["ok"] and d["calls"] == 4
    assert d["edges"]["gather->d2h"]["count"] == 12 and d["edges"]["gather->d2h"]["min_slack_us"] == 1000.0
    bad = tmp_path / "bad.jsonl"
    bad.write_text(json.dumps({"rank": 0, "phases": phases(late=1)}) + "\n")
    r = subprocess.run([sys.executable, HOST_ORDER, "--marks", str(bad)], capture_output=True, text=True)
    assert r.returncode == 1 and json.loads(r.stdout)["edges"]["gather->d2h"]["nviolations"] == 1
