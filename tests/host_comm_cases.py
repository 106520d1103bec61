"""The full-size cases on eight processes of a host-bootstrapped communicator -- TEST INFRASTRUCTURE shared by
tests/test_gpu_full_size.py (one pass) and tools/host_comm_stress.py (many, under diagnostic settings).

Every rank runs the same cases in the same order on cuda:0.  Around each case:
  * its own exchange buffer X is filled with a NaN poison (0xFF bytes) between two barriers, so a later read
    of a range nobody wrote in this case shows as "poison", not as the previous case's data;
  * after the case every rank fingerprints every rank's X as this process maps it, 2 MiB page by page
    (gpu_util.exchange_fingerprints), and the fingerprints are compared across ranks: a mapping that shows
    other memory than its owner's is named (viewer, owner, pages);
  * a wrong result is explained (whole_fold.explain): bad (block, piece) cells, runs, and what the values are.
Every rank reports; nothing stops at the first bad rank.
"""
import os

# (name, n, dtype, topology, peer form, host buffers)
CASES = [("c4_read", 1 << 28, "f32", "1", "read", False),
         ("c5_write", 1 << 29, "bf16", "8", "write", False),
         ("c4_host_read", 1 << 28, "f32", "1", "read", True),     # peer_allreduce_host, piece-pipelined
         ("c5_host_write", 1 << 29, "bf16", "8", "write", True)]  # whole bucket in, exchange, out
WIDE = [("c4_write", 1 << 28, "f32", "1", "write", False), ("c5_read", 1 << 29, "bf16", "8", "read", False)]
POISON = {"f32": 0xFFFFFFFF, "bf16": 0xFFFF}
HOST_PIECE_BYTES = 16 << 20   # the auto host piece at C4 (engine_host.cpp host_peer_piece): explain()'s unit


def inputs(P, n, tdt, seed, dev):
    import torch
    xs = []
    for r in range(P):
        gen = torch.Generator(device=dev)
        gen.manual_seed(seed + r)
        xs.append((torch.rand(n, generator=gen, device=dev) * 2 - 1).to(tdt))
    return xs


def worker(rank, world, port, q, cases, cycles=1, seed=6161, env=None):
    """One rank: `cycles` passes over `cases`; puts (rank, {"results": [...], "error": ...}) on q, one result
    per (cycle, case): name, cycle, ran (the form that ran), bad (whole_fold.explain or None), maps (mapping
    mismatches, [] if every page agrees), ms (the call's host time)."""
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "allreduce-over-mpi_amd"), os.path.join(root, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.update(env or {})
    import torch
    import torch.distributed as dist

    import ftar
    import ftar.dist
    import gpu_util
    import whole_fold
    out = {"results": []}
    if os.environ.get("FTAR_STRESS_PIDMAP"):   # tools/host_order_check.py: which trace is which rank
        with open(os.environ["FTAR_STRESS_PIDMAP"], "a") as f:
            f.write(f"{rank} {os.getpid()}\n")
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        comm = ftar.dist.init_host_comm(device=0)
        for cyc in range(cycles):
            for name, n, dt, topo, form, host in cases:
                tdt = {"f32": torch.float32, "bf16": torch.bfloat16}[dt]
                dist.barrier()                       # nobody reads my X any more
                gpu_util.poison_exchange(comm)
                dist.barrier()                       # everyone's X is poisoned before anyone starts
                xs = inputs(world, n, tdt, seed, dev)
                exp = whole_fold.fold(xs, n, "ring" if topo == "1" else "tree")
                x = xs[rank]
                xs.clear()
                comm.peer_direct = form
                marks = host and os.environ.get("FTAR_STRESS_MARKS") == "1"
                comm.phase_timing(marks)   # tools/host_order_check.py --marks: every hand-off's time
                t0 = time.perf_counter()
                if host:
                    h = x.cpu().pin_memory()
                    del x
                    comm.allreduce_host(None, h, n, dt, "sum", topo_=topo)
                    torch.cuda.synchronize()
                    ms = (time.perf_counter() - t0) * 1e3
                    y = h.to(dev)
                    del h
                else:
                    y = torch.empty_like(x)
                    comm.allreduce(x, y, n, dt, "sum", topo_=topo)
                    torch.cuda.synchronize()
                    ms = (time.perf_counter() - t0) * 1e3
                    del x
                glog = gather_forensics(comm, y, exp, tdt) if host and os.environ.get(
                    "FTAR_DEBUG_HOST_GATHER_LOG") == "1" else None
                ran = comm.last_exec()["form"]
                phases = comm.last_phases() if marks else None
                bad = None
                if whole_fold.first_mismatch(y, exp) is not None:
                    xs = inputs(world, n, tdt, seed, dev)
                    piece = HOST_PIECE_BYTES // (2 if dt == "bf16" else 4)
                    bad = whole_fold.explain(y, exp, xs, rank, "ring" if topo == "1" else "tree", piece,
                                             poison=POISON[dt])
                    if host:   # what this rank's exchange buffer holds there now: did the gather land?
                        bad["exchange_now"] = exchange_at(comm, bad, n, piece, tdt, exp, xs[rank], POISON[dt])
                    xs.clear()
                del y, exp
                torch.cuda.empty_cache()
                dist.barrier()                       # every rank's call and check are done: X is quiet
                fps = gpu_util.exchange_fingerprints(comm)
                allfp = [None] * world
                dist.all_gather_object(allfp, fps)
                maps = []
                for owner in range(world):
                    if owner == rank:
                        continue
                    pages = [i for i, (a, b) in enumerate(zip(fps[owner], allfp[owner][owner])) if a != b]
                    if pages or len(fps[owner]) != len(allfp[owner][owner]):
                        maps.append({"owner": owner, "pages": pages[:16], "npages": len(pages)})
                out["results"].append({"name": name, "cycle": cyc, "ran": ran, "bad": bad, "maps": maps,
                                       "ms": round(ms, 2), **({"phases": phases} if phases else {}),
                                       **({"gather_log": glog} if glog else {})})
                if rank == 0 and cycles > 1:
                    print(f"cycle {cyc} {name}: {ms:.1f} ms, {'BAD' if bad else 'ok'}", flush=True)
        dist.barrier()
        comm.destroy()
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001  report, don't hang the parent
        import traceback
        out["error"] = traceback.format_exc()
    q.put((rank, out))


def hw_fields(hw):
    """HW_REG_HW_ID (gfx9 layout) -> the fields that say where a wave ran."""
    return {"me": (hw >> 30) & 3, "pipe": (hw >> 6) & 3, "queue": (hw >> 24) & 7, "se": (hw >> 13) & 7,
            "cu": (hw >> 8) & 15}


def gather_forensics(comm, y, exp, tdt, read_dev=None):
    """The gather records of the last host call (FTAR_DEBUG_HOST_GATHER_LOG=1, engine_host.cpp log_gather):
    which workgroups left a record in host memory (not held in the GPU caches), how many times each workgroup
    id ran and on which XCDs (device-scope counters per id: 0 never, 2 handed out twice), on which XCD and
    hardware queue they ran, and -- when the result is wrong -- the same for the workgroups that own the wrong
    tiles (workgroup w copies tiles w / nsegs + j * grid / nsegs of segment w % nsegs).  Every piece is
    summarised; the bad ones are listed with their workgroups' records.  read_dev(ptr, words) -> numpy uint32
    reads the device records (2 words per workgroup; default: hipMemcpy)."""
    import collections
    import ctypes

    import numpy as np
    import torch

    iv = {torch.float32: torch.int32, torch.bfloat16: torch.int16}[tdt]
    esz = torch.tensor([], dtype=tdt).element_size()
    ne = y.view(iv) != exp.view(iv)
    if read_dev is None:
        import gpu_util
        hip = gpu_util.hip_runtime()

        def read_dev(ptr, words):
            buf = np.zeros(words, dtype=np.uint32)
            assert hip.hipMemcpy(ctypes.c_void_p(buf.ctypes.data), ctypes.c_void_p(ptr),
                                 ctypes.c_size_t(words * 4), 2) == 0
            return buf
    out = {"pieces": 0, "wgs": 0, "host_missing": 0, "dev_missing": 0, "runs": 0, "ids_run_twice": 0,
           "xcc_is_w_mod_8": 0, "queues": {}, "split_pieces": 0, "bad": []}
    k = 0
    while True:
        g = comm.gather_log(k)
        if g is None:
            break
        out["pieces"] = g["pieces"]
        grid, m, tile = g["grid"], g["nsegs"], g["tile_bytes"]
        devw = read_dev(g["dev_ptr"], 2 * grid)
        dev, dmask = devw[0::2], devw[1::2]
        h = g["host"]
        present_h = (h[:, 0] & 0x80000000) != 0
        present_d = dev != 0
        xcc = h[:, 0] & 15
        w = np.arange(grid)
        out["wgs"] += grid
        out["host_missing"] += int((~present_h).sum())
        out["dev_missing"] += int((~present_d).sum())
        out["runs"] += int(dev.astype(np.int64).sum())
        out["ids_run_twice"] += int((dev > 1).sum())
        out["xcc_is_w_mod_8"] += int((present_h & (xcc == w % 8)).sum())
        pq = collections.Counter("me{me}.pipe{pipe}.q{queue}".format(**hw_fields(int(hw)))
                                 for hw in h[present_h, 1])
        for key, c in pq.items():
            out["queues"][key] = out["queues"].get(key, 0) + c
        # one dispatch whose workgroups ran from more than one hardware queue slot: the queue was unmapped
        # (preempted) and mapped again part-way through the launch
        out["split_pieces"] += len(pq) > 1
        # the workgroups that own wrong tiles
        nb = grid // m
        te = tile // esz
        bad_w = collections.Counter()
        for j in range(m):
            lo, cnt = g["off"][j] // esz, g["bytes"][j] // esz
            seg = ne[lo:lo + cnt]
            nt = -(-cnt // te)
            pad = torch.zeros(nt * te, dtype=torch.bool, device=ne.device)
            pad[:cnt] = seg
            for t in torch.nonzero(pad.view(nt, te).any(1)).flatten().tolist():
                bad_w[(t % nb) * m + j] += 1
        if bad_w:
            ws = np.array(sorted(bad_w))
            t0 = int(h[present_h, 2].min()) if present_h.any() else 0
            span = (int(h[present_h, 3].max()) - t0) if present_h.any() else 0
            ends = [(int(h[x, 3]) - t0) for x in ws if present_h[x]]
            ph = np.nonzero(present_h)[0]
            starts = np.sort(h[ph, 2].astype(np.int64) - t0)
            gaps = np.diff(starts)
            out["bad"].append({
                "piece": k, "grid": grid, "nsegs": m, "bad_wgs": int(len(ws)), "bad_tiles": int(sum(bad_w.values())),
                "host_present": int(present_h[ws].sum()), "dev_present": int(present_d[ws].sum()),
                # workgroups that ran in this launch, counted by id: grid - bad_wgs if the missing ones never
                # ran, grid if their ids went to other workgroups (then some ids ran twice)
                "piece_runs": int(dev.astype(np.int64).sum()), "piece_ids_run_twice": int((dev > 1).sum()),
                # the ids that ran twice: their classes mod 8, and the XCD sets they ran on
                "twice_w_mod_8": dict(collections.Counter(int(x) % 8 for x in np.nonzero(dev > 1)[0])),
                "twice_xcds": dict(collections.Counter(
                    ",".join(str(b) for b in range(8) if int(mk) >> b & 1) for mk in dmask[dev > 1])),
                "xcc": dict(collections.Counter(int(x) for x in xcc[ws][present_h[ws]])),
                "w_mod_8": dict(collections.Counter(int(x) % 8 for x in ws)),
                "queues": dict(collections.Counter(
                    "me{me}.pipe{pipe}.q{queue}".format(**hw_fields(int(x))) for x in h[ws, 1][present_h[ws]])),
                "end_ticks_of_bad": [min(ends), max(ends)] if ends else None, "piece_span_ticks": span,
                "first_wgs": [int(x) for x in ws[:8]],
                # the piece's workgroups that did run: their queue slots, XCD - w mod 8 (the dispatch's
                # rotation over the XCDs), end times (percentiles 0/50/90/99/100) and the largest pause
                # between two consecutive workgroup starts, in wall-clock ticks (100 MHz)
                "piece_queues": dict(pq),
                "rotation": dict(collections.Counter(int(x) for x in (xcc[ph].astype(np.int64) - ph) % 8)),
                "end_pct": [int(v) for v in np.percentile(h[ph, 3].astype(np.int64) - t0, [0, 50, 90, 99, 100])]
                if len(ph) else None,
                "largest_start_gap": int(gaps.max()) if len(gaps) else None})
        k += 1
    return out


def exchange_at(comm, bad, n, piece, tdt, exp, mine, poison):
    """Classify what this rank's exchange buffer X holds, read afresh after the call, at the first bad cell's
    wrong elements: the final value (the gather's data is in X, so the D2H read it too early or stale), this
    rank's input (X still holds what the H2D put there), the poison, or other."""
    import ctypes

    import torch

    import gpu_util
    ptr, nbytes = comm.exchange_buffer(comm.rank)
    fc = bad["first_cell"]
    split = -(-n // comm.nranks)
    lo = fc["block"] * split + fc["piece"] * piece
    hi = min(n, fc["block"] * split + min(split, (fc["piece"] + 1) * piece))
    esz = torch.tensor([], dtype=tdt).element_size()
    if not ptr or hi * esz > nbytes:
        return None
    buf = torch.empty(hi - lo, dtype=tdt, device="cuda")
    hip = gpu_util.hip_runtime()
    assert hip.hipMemcpy(ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(ptr + lo * esz),
                         ctypes.c_size_t((hi - lo) * esz), 3) == 0
    torch.cuda.synchronize()
    iv = {torch.float32: torch.int32, torch.bfloat16: torch.int16}[tdt]
    xb, eb, mb = buf.view(iv), exp[lo:hi].view(iv), mine[lo:hi].view(iv)
    # the first cell's wrong elements: recompute them from the runs (explain keeps only counts)
    want = torch.zeros(hi - lo, dtype=torch.bool, device="cuda")
    for s0, ln in fc["runs"]:
        want[s0 - lo:s0 - lo + ln] = True
    pv = torch.tensor(poison, dtype=torch.int64).to(iv).to("cuda")
    return {"checked": int(want.sum().item()), "final": int((want & (xb == eb)).sum().item()),
            "own_input": int((want & (xb == mb) & (xb != eb)).sum().item()),
            "poison": int((want & (xb == pv)).sum().item())}


def run(cases, world=8, cycles=1, env=None, timeout=240):
    """Start `world` spawned ranks, return {rank: report}."""
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, world, port, q, cases, cycles, 6161, env)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        res = dict(q.get(timeout=timeout) for _ in range(world))
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    return res


def failures(res, world=8):
    """Every rank's problems, as lines: errors, wrong forms, wrong results (explained), bad mappings."""
    import whole_fold
    lines = []
    for r in range(world):
        rep = res.get(r, {"error": "no report"})
        if "error" in rep:
            lines.append(f"rank {r}: error: {rep['error']}")
        for x in rep.get("results", []):
            tag = f"rank {r} cycle {x['cycle']} {x['name']}"
            form = next(c[4] for c in CASES + WIDE if c[0] == x["name"])
            if x["ran"] != "peer-" + form:
                lines.append(f"{tag}: ran {x['ran']}")
            if x["bad"] is not None:
                lines.append(f"{tag}: {whole_fold.describe(x['bad'])}"
                             + (f"; exchange buffer there now: {x['bad']['exchange_now']}"
                                if x["bad"].get("exchange_now") else "")
                             + (f"; gather records of the bad pieces: {x['gather_log']['bad']}"
                                if x.get("gather_log") else ""))
            for mm in x["maps"]:
                lines.append(f"{tag}: mapping of rank {mm['owner']}'s exchange buffer differs from the owner's "
                             f"view in {mm['npages']} 2 MiB pages, first {mm['pages']}")
    return lines
