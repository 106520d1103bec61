#!/usr/bin/env python3
"""Benchmark of the FlexTree AllReduce hot path on MI355X (BASELINE.json metric).

  N = 1  (default) : the per-chunk k-way reduce-sum kernel alone, fp32,
                     k sources of 2^26 elements (256 MiB each) -> dst
                     (BASELINE configs[1]; the reference's vector_add.cu
                     harness, vector_add/vector_add.cu:49-170).
                     value = algorithmic HBM bytes (k+1)*n*4 per second.
  N > 1 (torchrun) : one process per GPU, RCCL p2p over xGMI, device-resident
                     fp32 bucket AllReduce (configs[2..3]; the reference's
                     benchmark.cpp harness, benchmark.cpp:155-167), default
                     2^28 elements (1 GiB) per rank, topology FT_TOPO/FT_LONELY
                     or the re-fitted cost model.
                     value = N * bucket bytes / t (aggregate algorithmic bandwidth).

Prints ONE JSON line on rank 0.  Inputs are synthetic (splitmix64 fp32 in
[-1, 1) at N=1, torch.rand at N>1) and resident in HBM before timing starts.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "allreduce-over-mpi_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBPS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
XGMI_LINK_GBPS = 76.8           # one xGMI link, one direction (153.6 GB/s bidirectional)
XGMI_LINKS = 7


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--sources", dest="k", type=int, default=2, help="N=1: number of source buckets k")
    ap.add_argument("--elements", dest="n", type=int, default=0, help="elements per bucket (default 2^26 at N=1, 2^28 at N>1)")
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--sets", type=int, default=4, help="N=1: disjoint buffer sets in rotation (1 = same buffers)")
    ap.add_argument("--topo", default=None, help="N>1: FT_TOPO string (default: env FT_TOPO, else cost model)")
    ap.add_argument("--lonely", type=int, default=0)
    ap.add_argument("--chunk-bytes", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="N=1: CPU baseline sample length")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-peer", action="store_true", help="N>1: leave the peer-direct forms out of the sweep")
    ap.add_argument("--sweep", action="store_true", help="N=1: also report k=1..16 (vector_add.cu:182)")
    ap.add_argument("--no-engine-local", action="store_true",
                    help="N=1: skip the engine_local line item (P = 8 in-process ranks on this GPU at the C4 bucket)")
    ap.add_argument("--no-host-local", action="store_true",
                    help="N=1: skip the host_local line item (P = 2 in-process ranks, pinned host buckets of C3)")
    ap.add_argument("--save-cost", default="",
                    help="N>1: write the execution model's constants re-fitted on this node to this calibration "
                         "file (rank 0; load it with FTAR_COST_FILE so every later MPI_Allreduce_FT prices with them)")
    ap.add_argument("--engine-local-only", action="store_true",
                    help="run only the engine_local line item (for a kernel trace of it) and print it")
    ap.add_argument("--force-dist", action="store_true", help="take the torchrun/RCCL path even at WORLD_SIZE=1")
    ap.add_argument("--no-c5", action="store_true", help="N>1: skip the bf16 configs[4] line item")
    ap.add_argument("--elements-c5", dest="n_c5", type=int, default=0, help="N>1: bf16 elements (default 2^29)")
    ap.add_argument("--no-host", action="store_true", help="N>1: skip the host-memory end-to-end line item")
    ap.add_argument("--host-comm", action="store_true",
                    help="N>1 rehearsal on fewer GPUs than ranks: communicator bootstrapped over gloo "
                         "(ftar_comm_init_host, no RCCL), ranks may share a GPU, peer-direct forms only")
    ap.add_argument("--rccl-loopback", action="store_true",
                    help="N>1 rehearsal on fewer GPUs than ranks over RCCL itself: every rank gets its own "
                         "NCCL_HOSTID, so RCCL accepts ranks sharing a GPU and moves ncclSend/ncclRecv over "
                         "loopback sockets (every RCCL form runs; timings are not xGMI numbers)")
    return ap.parse_args()


KERNEL_SOURCES = ("allreduce-over-mpi_amd/csrc/reduce_impl.h", "allreduce-over-mpi_amd/csrc/reduce_kernels.hip")


def kernel_source_digest(root=ROOT):
    """sha256 (16 hex digits) of the reduce kernels' sources: a PMC measurement belongs to the kernels
    these sources compile to, so bench.py and tools/pmc_summary.py both stamp it."""
    import hashlib
    h = hashlib.sha256()
    for rel in KERNEL_SOURCES:
        with open(os.path.join(root, rel), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def pmc_traffic(workload, kernel, summary=None):
    """Per-launch HBM bytes of `workload` measured with rocprofv3 --pmc (profiles/pmc_summary.json) -- only
    when that measurement was taken on the kernel this run launched (same template id, same kernel sources).
    Returns (bytes or None, provenance dict): a measurement of another kernel is never reported as this one's."""
    p = summary or os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(p) as f:
            e = json.load(f).get(workload)
    except (OSError, ValueError):
        e = None
    if not e:
        return None, {"traffic_note": f"no PMC measurement of {workload} in profiles/pmc_summary.json"}
    digest = kernel_source_digest()
    src = {"file": "profiles/pmc_summary.json", "kernel": e.get("kernel"), "commit": e.get("commit"),
           "kernel_sources_sha": e.get("kernel_sources_sha"), "profiles": e.get("source")}
    if e.get("kernel") != kernel:
        return None, {"traffic_note": f"the PMC summary measured {e.get('kernel')}; this run launched {kernel}",
                      "traffic_source": src}
    if e.get("kernel_sources_sha") != digest:
        return None, {"traffic_note": f"the PMC summary was taken on kernel sources {e.get('kernel_sources_sha')}; "
                                      f"this tree's are {digest}", "traffic_source": src}
    return e.get("hbm_bytes_per_launch"), {"traffic_source": src}


def host_cores():
    """The CPU this process may actually use: its affinity set and its cgroup quota (cpu.max, v2; cfs
    quota/period, v1), next to the machine's count.  os.cpu_count() counts the whole machine, which on a
    shared GPU box is many times the share a job gets."""
    info = {"machine_cpus": os.cpu_count()}
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["affinity_cpus"] = None
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                per = int(f.read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    info["cgroup_quota_cpus"] = round(quota, 2) if quota else None
    avail = [v for v in (info["affinity_cpus"], quota) if v]
    info["available_cpus"] = round(min(avail), 2) if avail else info["machine_cpus"]
    return info


def cpu_baseline(k, n, seconds):
    """The reference's reduce_sum<float> (mpi_mod.hpp:812, 14 OpenMP threads, :820) on this host,
    built from the unmodified header into oracle/_ref/ref_golden; else the oracle port.  `cores` = the
    threads it ran; `cores_available` = what this process may use (affinity, cgroup quota).  Two legs of
    half the time each: `value` is the warm leg (the same buffers every call, as the reference's own
    harness reruns them) and its best call; `rotated` is the cold leg (2 disjoint buffer sets in turn, the
    regime of the GPU line's rotated sets, bench_single), best and median."""
    ref = os.path.join(ROOT, "oracle", "_ref", "ref_golden")
    hc = host_cores()
    if os.path.exists(ref):
        try:
            def leg(sets, secs):
                out = subprocess.run([ref, "bench", "--k", str(k), "--n", str(n), "--seconds", str(secs), "--sets",
                                      str(sets)], capture_output=True, text=True, timeout=secs * 6 + 120,
                                     check=True).stdout
                return json.loads(out.strip().splitlines()[-1])
            d = leg(1, seconds / 2)
            r = leg(2, seconds / 2)
            return {"value": round(d["GBps_best"], 3), "unit": "GB/s", "cores": d["threads"], "kind": "reference",
                    "buffers": "same every call (warm)", "statistic": "best",
                    "median": round(d["GBps_median"], 3), "mean": round(d["GBps_mean"], 3), "samples": d["iters"],
                    "rotated": {"buffers": "2 disjoint sets in turn (cold, as the GPU line)", "best": round(r["GBps_best"], 3),
                                "median": round(r["GBps_median"], 3), "samples": r["iters"]},
                    "cores_available": hc,
                    "sample": f"FlexTree::reduce_sum<float> k={k} n={n} fp32, the same buffers every call: best of "
                              f"{d['iters']} calls in ~{seconds / 2:.0f}s (median {d['GBps_median']:.2f}); 2 rotated "
                              f"sets: best {r['GBps_best']:.2f}, median {r['GBps_median']:.2f} of {r['iters']} calls; "
                              f"{d['threads']} OpenMP threads (mpi_mod.hpp:820) on {hc['available_cpus']} available "
                              f"CPUs (affinity {hc['affinity_cpus']}, cgroup quota {hc['cgroup_quota_cpus']}, "
                              f"machine {hc['machine_cpus']})"}
        except Exception as e:  # fall through to the port
            sys.stderr.write(f"reference cpu baseline failed: {e}\n")
    import numpy as np
    import oracle_lib
    from ftar import inputs as fi
    m = min(n, 1 << 24)
    xs = [fi.fill("f32", 0x5EED, j, m) for j in range(k)]
    out = np.empty(m, np.float32)
    times, t_end = [], time.time() + seconds
    while time.time() < t_end or not times:
        t0 = time.perf_counter()
        oracle_lib.reduce(6, 0, xs, out=out)
        times.append(time.perf_counter() - t0)
    times.sort()
    best, med, iters = times[0], times[len(times) // 2], len(times)
    return {"value": round((k + 1) * m * 4 / best / 1e9, 3), "unit": "GB/s", "cores": 1, "kind": "port",
            "buffers": "same every call (warm)", "statistic": "best",
            "median": round((k + 1) * m * 4 / med / 1e9, 3), "samples": iters,
            "cores_available": hc,
            "sample": f"oracle reduce k={k} n={m} fp32 single thread, best of {iters}"}


def bench_single(a):
    """N = 1: the k-way reduce kernel on `sets` disjoint (k sources + destination) buffer sets, one step per
    set in rotation, so every launch streams data the previous launches did not leave in the 256 MB
    Infinity Cache (MALL): the AllReduce's regime, where every piece is new data.  The same-buffer loop of
    the reference harness (vector_add.cu:110-140) is reported next to it as `same_buffers`: there the MALL
    absorbs part of the rewritten destination and the rate overstates HBM."""
    import numpy as np
    import torch

    import ftar
    from ftar import inputs as fi

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    k, n = a.k, a.n or (1 << 26)
    esz = ftar.dtype_size(a.dtype)
    sets = max(1, a.sets)
    m = min(n, 1 << 16)
    srcs, dsts, probes = [], [], []
    for i in range(sets):
        ss, heads, tails = [], [], []
        for j in range(k):
            x = fi.fill(a.dtype, 0x5EED + i, j, n)
            ss.append(torch.from_numpy(x.view(np.uint8)).to(dev))
            heads.append(x[:m].copy())
            tails.append(x[n - m:].copy())
            del x
        srcs.append(ss)
        dsts.append(torch.empty(n * esz, dtype=torch.uint8, device=dev))
        probes.append((heads, tails))
    stream = torch.cuda.current_stream()
    ptrs = [[t.data_ptr() for t in ss] for ss in srcs]

    def step(i):
        ftar.reduce(ptrs[i % sets], dsts[i % sets].data_ptr(), n, a.dtype, "sum", stream=stream)

    def run(steps, warmup, rotate):
        for i in range(warmup):
            step(i if rotate else 0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        for i in range(steps):
            step(i if rotate else 0)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / steps, time.perf_counter() - t0   # one kernel per step, same stream

    ms, wall = run(a.steps, a.warmup, rotate=True)
    kernel = ftar.last_kernel()   # the kernel those launches ran (the PMC traffic must be this one's)
    ms_same, _ = run(a.steps, a.warmup, rotate=False)
    algo_bytes = (k + 1) * n * esz
    gbps = algo_bytes / (ms * 1e-3) / 1e9
    gbps_same = algo_bytes / (ms_same * 1e-3) / 1e9
    for i in range(sets):   # every set's destination holds its last reduce
        step(i)
    torch.cuda.synchronize()

    # spot check of every set (first and last 64 Ki elements): numpy's fp32 adds, folded left to right
    # like reduce_sum (mpi_mod.hpp:856-863), must match bit for bit
    check = "skipped"
    if a.dtype == "f32":
        ok = True
        for i in range(sets):
            got = dsts[i].view(torch.float32)
            for part, lo in ((0, 0), (1, n - m)):
                parts = probes[i][part]
                exp = parts[0].copy()
                for h in parts[1:]:
                    exp = (exp + h).astype(np.float32)
                g = got[lo:lo + m].cpu().numpy()
                ok &= bool(np.array_equal(g.view(np.uint32), exp.view(np.uint32)))
        check = "bit-exact" if ok else "MISMATCH"

    workload = f"reduce_k{k}_{a.dtype}_n{n}"
    traffic, prov = pmc_traffic(workload, kernel)
    res = {
        "metric": "fp32 bucket reduce-sum GB/s (device-resident) at 1/2/4/8 MI355X",
        "value": round(gbps, 2), "unit": "GB/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(ms, 5), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": a.dtype, "data": f"synthetic (splitmix64 uniform [-1,1), HBM-resident, {sets} buffer sets in rotation)",
        "config": {"workload": "1xMI355X local k-way reduce-sum kernel (BASELINE configs[1])", "k": k,
                   "elements_per_bucket": n, "bucket_bytes": n * esz, "algorithmic_bytes_per_step": algo_bytes,
                   "buffer_sets": sets},
        "roofline": {"bound": "hbm", "achieved": round(gbps, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(gbps / HBM_PEAK_GBPS, 4), "traffic": traffic, "kernel": kernel,
                     "kernel_sources_sha": kernel_source_digest(), **prov},
        "same_buffers": {"GBps": round(gbps_same, 2), "ms_per_step": round(ms_same, 5),
                         "note": "every step on set 0 (the reference harness's loop); the Infinity Cache absorbs "
                                 "part of the rewritten destination, so this overstates HBM"},
        "check": check, "wall_s": round(wall, 4),
    }
    # vector_add.cu:182: k = 1..16 with --sweep; by default k = 8 only (k in {2, 8}); two sets in
    # rotation (each (k+1) x 256 MiB >> the MALL)
    sweep = {}
    for kk in (range(1, 17) if a.sweep else (8,)):
        sw = [[torch.empty_like(srcs[0][0]).copy_(srcs[i % sets][j % k]) for j in range(kk)] for i in range(2)]
        sd = [torch.empty_like(dsts[0]) for _ in range(2)]
        pp = [[t.data_ptr() for t in w] for w in sw]
        for i in range(2):
            ftar.reduce(pp[i], sd[i].data_ptr(), n, a.dtype, "sum", stream=stream)
        torch.cuda.synchronize()
        reps = 6 if a.sweep else 20

        def timed_k(dst_of):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i in range(reps):
                ftar.reduce(pp[i % 2], dst_of(i % 2), n, a.dtype, "sum", stream=stream)
            e1.record(stream)
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / reps
        t = timed_k(lambda i: sd[i].data_ptr())
        kern = ftar.last_kernel()
        bw = (kk + 1) * n * esz / (t * 1e-3) / 1e9
        tr, pv = pmc_traffic(f"reduce_k{kk}_{a.dtype}_n{n}", kern)
        sweep[kk] = {"ms": round(t, 4), "GBps": round(bw, 1), "frac": round(bw / HBM_PEAK_GBPS, 4),
                     "kernel": kern, "traffic": tr, **pv}
        if kk == 8 and not a.sweep:
            # in place (destination = source 0): the width-8 tree's fold in an MPI_IN_PLACE AllReduce, whose own
            # block is operand and result; same bytes, (k+1) x n x 4 (the values grow; timing only)
            ti = timed_k(lambda i: pp[i][0])
            bwi = (kk + 1) * n * esz / (ti * 1e-3) / 1e9
            sweep[kk]["in_place"] = {"ms": round(ti, 4), "GBps": round(bwi, 1), "frac": round(bwi / HBM_PEAK_GBPS, 4)}
        del sw, sd
    res["k_sweep" if a.sweep else "k8"] = sweep if a.sweep else sweep[8]
    del srcs, dsts, sweep
    if not a.no_engine_local:
        torch.cuda.empty_cache()
        try:
            res["engine_local"] = engine_local(steps=5, warmup=2)
        except Exception as e:   # a line item: its failure must not cost the headline
            res["engine_local"] = {"error": str(e)[:300]}
    if not a.no_host_local:
        torch.cuda.empty_cache()
        try:
            res["host_local"] = host_local()
        except Exception as e:   # a line item: its failure must not cost the headline
            res["host_local"] = {"error": str(e)[:300]}
    if not a.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(k, n, a.cpu_seconds)
    print(json.dumps(res), flush=True)


def plan_hbm_bytes(ftar, topo, world, count, esz, allgather="direct", reduce_scatter="direct"):
    """HBM bytes one AllReduce call moves on ONE device when all `world` ranks share it (the in-process
    transport): every received block is one device copy (read + write), every fold reads its k sources and
    writes its block.  From the plans themselves (ftar_plan_json), summed over the ranks."""
    total = 0
    for r in range(world):
        p = ftar.plan_json(topo, world, r, count, allgather, reduce_scatter)
        for st in p["stages"]:
            total += sum(2 * x[3] for x in st["recvs"]) * esz
            total += sum((len(red["srcs"]) + 1) * red["len"] for red in st["reduces"]) * esz
    return total


def engine_local(steps=5, warmup=2, world=8, n=1 << 28, topo="8", chunk_bytes=None):
    """The engine itself on this one GPU, against HBM: P = 8 in-process ranks (the
    local transport, one host thread per rank, its transfers device copies on the comm streams) run the C4
    bucket -- 2^28 fp32 per rank, tree(8) in the direct form, the execution model's piece -- through the
    same two-stream executor as over RCCL (mpi_mod.hpp:1689-1715 is the per-step loop it replaces).  Rate =
    the HBM bytes the call moves (gather copies + 8-way folds + all-gather copies, from the plans) / the
    call's time, against 8 TB/s: how close the whole pipeline, copies and folds overlapped on two streams
    per rank, comes to the memory roofline.  Checked bit-exact against the direct fold on a sample."""
    import numpy as np
    import torch

    import ftar
    dev = torch.device("cuda:0")
    esz = 4
    ch = ftar.exec_choose(world, n * esz, topo_=topo, form="direct", chunk_bytes=chunk_bytes)
    g = ftar.Comm.init_local(world)
    try:
        g.set_form("direct")
        g.set_chunk_bytes(ch.chunk_bytes or (n // world) * esz)   # 0 (whole blocks): one piece per block
        gen = torch.Generator(device=dev)
        gen.manual_seed(0xC4)
        xs = [torch.rand(n, device=dev, generator=gen) * 2 - 1 for _ in range(world)]
        ys = [torch.empty_like(x) for x in xs]
        stream = torch.cuda.current_stream()
        streams = [stream] * world

        def call():
            g.allreduce(xs, ys, n, "f32", "sum", topo_=topo, streams=streams)
        for _ in range(warmup):
            torch.cuda._sleep(64)   # a marker kernel between calls for the trace (tools/engine_local_trace.py)
            call()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        per = []
        t0 = time.perf_counter()
        for _ in range(steps):
            torch.cuda._sleep(64)
            torch.cuda.synchronize()
            e0.record(stream)
            call()
            e1.record(stream)
            torch.cuda.synchronize()
            per.append(e0.elapsed_time(e1))
        wall = time.perf_counter() - t0
        ms = sorted(per)[len(per) // 2]
        # sample check: tree(8)'s fold of block b is the owner's copy first, then the peers in ascending
        # rank (mpi_mod.hpp:1316-1358), i.e. ((x_b + x_0) + x_1) + ... skipping b
        split = n // world
        idx = torch.randint(0, n, (4096,), device=dev, generator=gen)
        owner = idx // split
        acc = torch.stack([x[idx] for x in xs])            # [P, m]
        want = acc.gather(0, owner.unsqueeze(0)).squeeze(0).clone()
        for q in range(world):
            want = torch.where(owner == q, want, want + acc[q])
        ok = all(bool(torch.equal(y[idx].view(torch.int32), want.view(torch.int32))) for y in ys)
        hbm = plan_hbm_bytes(ftar, topo, world, n, esz)
        gbps = hbm / (ms * 1e-3) / 1e9
        whole = None
        if chunk_bytes is None:   # the same calls with whole blocks (one piece per block): nothing to overlap
            g.set_chunk_bytes(split * esz)   # on one GPU, where every copy and fold shares the one HBM
            call()
            wper = []
            for _ in range(steps):
                torch.cuda.synchronize()
                e0.record(stream)
                call()
                e1.record(stream)
                torch.cuda.synchronize()
                wper.append(e0.elapsed_time(e1))
            wms = sorted(wper)[len(wper) // 2]
            whole = {"chunk_bytes": split * esz, "ms_median": round(wms, 4),
                     "hbm_frac": round(hbm / (wms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                     "model_ms": round(ftar.exec_choose(world, n * esz, topo_=topo, form="direct",
                                                        chunk_bytes=split * esz).seconds * 1e3, 4)}
        peer = None
        if chunk_bytes is None:
            # the peer-read form on registered buffers, the IPC form a node may pick: the fold reads the 8
            # inputs where they lie, the gather pulls the 7 final blocks -- no scratch pass: 9 + 14 block
            # passes per rank instead of 37 (the same kernels read peers' HBM over xGMI on a node)
            ids = g.register(xs, n * esz) + g.register(ys, n * esz)
            try:
                g.set_peer_direct("read")
                call()
                pper = []
                for _ in range(steps):
                    torch.cuda._sleep(64)   # markers: the last `steps` calls of a trace are these
                    torch.cuda.synchronize()
                    e0.record(stream)
                    call()
                    e1.record(stream)
                    torch.cuda.synchronize()
                    pper.append(e0.elapsed_time(e1))
                pms = sorted(pper)[len(pper) // 2]
                pbytes = world * ((world + 1) + 2 * (world - 1)) * split * esz
                pok = all(bool(torch.equal(y[idx].view(torch.int32), want.view(torch.int32))) for y in ys)
                ran = g.comms[0].last_exec()["form"]
                peer = {"form": ran, "ms_median": round(pms, 4), "hbm_bytes_per_call": pbytes,
                        "hbm_GBps": round(pbytes / (pms * 1e-3) / 1e9, 1),
                        "hbm_frac": round(pbytes / (pms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                        "check": "bit-exact (the same sample)" if pok else "MISMATCH"}
            finally:
                g.set_peer_direct(0)
                g.deregister(ids[:world])
                g.deregister(ids[world:])
        return {"workload": f"P = {world} in-process ranks on one MI355X, tree({topo}) direct, C4 bucket "
                            f"(2^28 fp32 per rank), " + ("the model's piece" if chunk_bytes is None else "piece fixed"),
                "ranks": world, "elements_per_rank": n, "topology": topo, "form": "direct",
                "chunk_bytes": ch.chunk_bytes, "model": ch.as_dict(), "ms_median": round(ms, 4),
                "ms_all": [round(x, 4) for x in per], "wall_s": round(wall, 3),
                "hbm_bytes_per_call": hbm, "hbm_GBps": round(gbps, 1), "hbm_peak_GBps": HBM_PEAK_GBPS,
                "hbm_frac": round(gbps / HBM_PEAK_GBPS, 4), "check": "bit-exact (4096-element sample, every rank)"
                if ok else "MISMATCH", "whole_blocks": whole, "peer_read_registered": peer,
                "note": "HBM bytes from the plans: every received block one device copy (read + write), every "
                        "fold k sources + 1 destination; all 8 ranks' copies and folds share this GPU's HBM. "
                        "ms = events around the group call on the ranks' stream (the call returns once every "
                        "rank's work is enqueued; the enqueue itself is inside the events)"}
    finally:
        g.destroy()


def host_local(steps=10, warmup=1, world=2, n=1 << 26, topo="2"):
    """The reference's own setting on this one GPU (MPI_Allreduce_FT on host buffers,
    mpi_mod.hpp:1723-1778, benchmark.cpp:125-131): P = 2 in-process ranks, a pinned host bucket each (the C3
    bucket, 2^26 fp32 = 256 MiB), ftar_allreduce_host_group -- H2D, the exchange and D2H pipelined per piece,
    the path MPI_Allreduce_FT takes.  Both ranks' copies share this GPU's one PCIe link (on a node each rank
    has its own).  The call returns once the host buckets hold the result: wall time.  Checked bit-identical
    to the device path on the same inputs."""
    import torch

    import ftar
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev)
    gen.manual_seed(0xC3)
    xd = [torch.rand(n, device=dev, generator=gen) * 2 - 1 for _ in range(world)]
    hx = [x.cpu().pin_memory() for x in xd]
    hy = [torch.empty_like(h).pin_memory() for h in hx]
    g = ftar.Comm.init_local(world)
    try:
        g.set_form("direct")

        def call():
            g.allreduce(hx, hy, n, "f32", "sum", topo_=topo, host=True)
        for _ in range(warmup):
            call()
        per = []
        for _ in range(steps):
            t0 = time.perf_counter()
            call()
            per.append((time.perf_counter() - t0) * 1e3)
        ms = sorted(per)[len(per) // 2]
        best = min(per)
        yd = [torch.empty_like(x) for x in xd]
        g.allreduce(xd, yd, n, "f32", "sum", topo_=topo)   # the device path, same inputs and plan
        torch.cuda.synchronize()
        same = all(torch.equal(hy[r], yd[r].cpu()) for r in range(world))
        bucket = n * 4
        return {"workload": f"P = {world} in-process ranks on one MI355X, pinned host buckets of 2^26 fp32 "
                            f"(C3), tree({topo}) direct, ftar_allreduce_host_group (the MPI_Allreduce_FT path)",
                "ranks": world, "elements_per_rank": n, "ms_median": round(ms, 3), "ms_best": round(best, 3),
                "ms_all": [round(x, 3) for x in per],
                "algbw_GBps_per_rank": round(bucket / (ms * 1e-3) / 1e9, 2),
                "algbw_GBps_per_rank_best": round(bucket / (best * 1e-3) / 1e9, 2),
                "pcie_GBps_both_directions": round(2 * world * bucket / (ms * 1e-3) / 1e9, 2),
                "check": "bit-identical to the device path" if same else "MISMATCH",
                "note": "both ranks' H2D and D2H share this GPU's one PCIe link (57 GB/s per direction alone, "
                        "48.6 each with both at once, DESIGN §6); with one rank per GPU each has its own"}
    finally:
        g.destroy()


def reference_mpi_path(world, n=1 << 24, repeat=20, seconds=150):
    """The reference's MPI_Allreduce_FT (ring, FT_TOPO=1: its own cost model's choice at P = 2, 4, 8) with
    `world` MPI ranks on this host, fp32 bucket of n elements (a bounded sample of the 1 GiB workload),
    built from the unmodified header into oracle/_ref/ref_golden.  None when the binary or MPICH is absent."""
    ref = os.path.join(ROOT, "oracle", "_ref", "ref_golden")
    mpiexec = "/opt/conda/bin/mpiexec"
    if world < 2 or not (os.path.exists(ref) and os.path.exists(mpiexec)):
        return None   # P = 1 is the reference's memcpy (mpi_mod.hpp:1739), nothing to time
    env = dict(os.environ, FT_TOPO="1")
    for k in list(env):   # a clean MPI job: not the torchrun rank's rendezvous variables
        if k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK") or k.startswith("TORCHELASTIC"):
            env.pop(k)
    try:
        p = subprocess.run([mpiexec, "-n", str(world), ref, "arbench", "--n", str(n), "--repeat", str(repeat)],
                           capture_output=True, text=True, timeout=seconds, env=env)
        d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
        hc = host_cores()
        d["cores"] = world * 14   # 14 OpenMP threads per rank, hard-coded (mpi_mod.hpp:820)
        d["cores_available"] = hc
        d["sample"] = (f"{world} MPI ranks on the host, ring (FT_TOPO=1), {n} fp32 per rank, best of {repeat} "
                       f"timed calls (benchmark.cpp timing: Barrier + Wtime, max over ranks); {world} x 14 OpenMP "
                       f"threads on {hc['available_cpus']} available CPUs")
        return d
    except Exception as e:  # noqa: BLE001  a baseline must not cost the run its line
        return {"error": str(e)[:200]}


def sample_index(n, dev, m=4096):
    """m element indices spread over [0, n), computed in int64.  (A float32 linspace rounds n - 1 up to n
    once n > 2^24 -- at 2^28 elements it indexes one past the end of the bucket.)"""
    import torch
    m = max(1, min(m, n))
    idx = torch.arange(m, dtype=torch.int64, device=dev) * (n - 1) // max(1, m - 1)
    assert int(idx[-1]) <= n - 1 and int(idx[0]) >= 0
    return idx


def link_rate_from_probe(probe, world):
    """Per-link, per-direction GB/s measured by ftar_xgmi_probe (every rank copying at once, so each link
    carries one direction per mode): the best of read/write from one peer and of read/write from all
    peers divided by the P-1 links they spread over.  None when the probe did not run or measured nothing."""
    if not probe or world < 2:
        return None
    rates = []
    for key, per in (("read_one_peer", 1), ("write_one_peer", 1), ("read_all_peers", world - 1),
                     ("write_all_peers", world - 1), ("dma_read_all_peers", world - 1),
                     ("dma_write_all_peers", world - 1)):
        v = probe.get(key)
        if isinstance(v, (list, tuple)):   # bench line form: [min, max] over ranks -> the slowest rank
            v = v[0]
        if isinstance(v, (int, float)) and v > 0:
            rates.append(v / per)
    return max(rates) if rates else None


XGMI_CONVENTION = ("achieved = busBW = algBW x 2(P-1)/P: the bytes one rank sends (and, at the same time, "
                   "receives) per second; peak = links x 76.8 GB/s, the ONE-direction rate of a 153.6 GB/s "
                   "bidirectional xGMI link")


def allreduce_roofline(world, gpus, bucket, ms, links, probe_link_gbps=None):
    """Roofline object of one N>1 AllReduce line (ms per call, bucket bytes per rank).

    - P = 1: nothing crosses a link; the call is one pass over the bucket (read + write), so the bound is
      HBM and achieved = 2 * bucket / t.
    - ranks sharing GPUs (the --host-comm rehearsal): neither an xGMI nor a per-GPU HBM figure; None.
    - P > 1: busBW = algBW * 2(P-1)/P (bytes each rank sends, and receives, per second) against the SPEC
      peak, links x 76.8 GB/s per direction (153.6 GB/s bidirectional).  The xGMI probe's measured per-link
      rate, when the run has one, only gives a second ratio, `frac_of_probe`: a slow or under-driven probe
      must not flatter `frac`.
    Never returns a frac outside (0, 1]: a denominator the work exceeds does not describe it, and the
    object then carries frac None and says why."""
    if ms <= 0 or bucket <= 0:
        return None
    algbw = bucket / (ms * 1e-3) / 1e9
    if world == 1:
        ach = 2 * algbw
        return {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBPS, 4), "traffic": None,
                "note": "P=1: the AllReduce is one local pass over the bucket (read + write), no link crossed"}
    if world > gpus:
        return None
    busbw = algbw * 2 * (world - 1) / world
    links = max(1, min(XGMI_LINKS, links))
    peak = links * XGMI_LINK_GBPS
    res = {"bound": "xgmi", "achieved": round(busbw, 2), "peak": round(peak, 2), "unit": "GB/s",
           "frac": round(busbw / peak, 4) if busbw <= peak else None, "traffic": None,
           "direction_convention": XGMI_CONVENTION,
           "note": f"busBW vs {links} xGMI link(s) x {XGMI_LINK_GBPS} GB/s per direction (spec)"}
    if busbw > peak:
        res["note"] = (f"busBW exceeds {links} link(s) x {XGMI_LINK_GBPS} GB/s per direction: the link count "
                       "does not describe this run's data movement; no fraction reported")
    if probe_link_gbps and probe_link_gbps > 0:
        res["probe_peak"] = round(links * probe_link_gbps, 2)
        res["frac_of_probe"] = round(busbw / (links * probe_link_gbps), 4)
        res["probe_note"] = (f"{links} link(s) x {probe_link_gbps:.1f} GB/s, the per-link one-direction rate "
                             "ftar_xgmi_probe measured in this run (a ratio to what copy kernels reached, not "
                             "to the hardware)")
    return res


def links_driven(world, topology, form):
    """xGMI links one rank drives at once: every peer in the one-round forms (direct, collective, peer);
    in the reference's rounds ("stages"), one neighbour (ring) or the widest stage's group (tree).
    `topology` is the str() of a Topo ("ring", "2,4", "2,2+1")."""
    if form.split(":")[0] != "stages":
        return min(XGMI_LINKS, world - 1)
    if topology == "ring":
        return 1
    widths = [int(w) for w in topology.split("+")[0].split(",")]
    return min(XGMI_LINKS, max(widths) - 1)


def probe_cap_entries(probe, by_cap, gain=1.10):
    """Sweep entries for the peer forms' copy-kernel cap: ftar_xgmi_probe measured read/write from all peers
    uncapped ([min, max] over ranks) and at 4..64 workgroups per peer (min over ranks).  For each direction
    whose best capped rate beats the uncapped minimum by `gain`, the registered peer form of that direction
    with that cap ("peer-read-reg:wgN" / "peer-write-reg:wgN")."""
    out = []
    for key, form in (("read_all_peers", "peer-read-reg"), ("write_all_peers", "peer-write-reg")):
        base = probe.get(key)
        base = base[0] if isinstance(base, (list, tuple)) else base
        rates = {int(w): v.get(key, 0) for w, v in (by_cap or {}).items()}
        if not base or not rates:
            continue
        w, r = max(rates.items(), key=lambda kv: kv[1])
        if r > gain * base:
            out.append(f"{form}:wg{w}")
    return out


RCCL_P2P_FORMS = ("direct", "stages")   # ncclSend/ncclRecv both ways ("collective" ends in ncclAllGather)


def rccl_p2p_best(sweep, world, gpus, bucket, links_of):
    """The fastest validated sweep entry whose data moved by RCCL point-to-point (north_star's transport:
    ncclSend/ncclRecv, forms "direct", "direct:ncclreg", "stages"), with its roofline -- reported next to the
    headline, which may be an IPC peer form, so the RCCL path is graded on its own.  links_of(entry) gives the
    links one rank drives in that entry's form.  None when no such entry validated."""
    ok = [r for r in sweep if "ms" in r and r.get("check") == "ok" and r.get("form", "").split(":")[0] in RCCL_P2P_FORMS]
    if not ok:
        return None
    b = min(ok, key=lambda r: r["ms"])
    alg = bucket / (b["ms"] * 1e-3) / 1e9
    return {"topology": b["topology"], "chunk_bytes": b["chunk_bytes"], "form": b["form"],
            "form_label": form_label(b["topology"], b["form"]), "ms": b["ms"],
            "algbw_GBps_per_rank": round(alg, 2),
            "busbw_GBps_per_rank": round(alg * 2 * (world - 1) / world if world > 1 else alg, 2),
            "roofline": allreduce_roofline(world, gpus, bucket, b["ms"], links_of(b)),
            "note": "fastest validated sweep entry moved by RCCL ncclSend/ncclRecv (sweep timing: "
                    "min(5, steps) calls after 1 warmup)"}


def form_label(topology, form):
    """What a form string ran, in words (a gather must not read as a ring): the one-round
    "direct" form gathers every copy of a block at its owner and folds them there in the topology's own
    order -- the ring's hop order on FT_TOPO=1, same bits as the reference ring, tree(8)'s bytes over all
    links -- while "stages" replays the reference's own rounds (the ring's 2(P-1) neighbour steps, one link
    each)."""
    base, _, tune = form.partition(":")
    reg = base.endswith("-reg")
    base = base[:-4] if reg else base
    ring = str(topology) in ("ring", "1")
    order = "ring-order" if ring else "tree-order"
    lab = {"direct": f"direct (gather + {order} fold)",
           "stages": "stages (reference ring steps)" if ring else "stages (reference tree stages)",
           "collective": f"collective (gather + {order} fold, ncclAllGather)",
           "peer-read": f"peer-read (IPC loads over xGMI + {order} fold)",
           "peer-write": f"peer-write (IPC stores over xGMI + {order} fold)",
           "auto": "auto (the execution model's form per call)"}.get(base, base)
    if reg:
        lab += " on registered buffers"
    if tune:
        lab += f" [{tune}]"
    return lab


def c4_ring_by_form(sweep, world, gpus, bucket, links_of):
    """BASELINE configs[3] (ring AllReduce, chunk size swept): the fastest validated ring entry of each RCCL
    p2p form, with its label, the pieces swept and its roofline.  `judged` marks the form the >= 70 % xGMI
    busBW target is judged on: direct -- the reference ring's association order, tree(P)'s data
    movement on every link; the staged ring is single-link bound by construction (its roofline is 1 link)."""
    out = {}
    for form in RCCL_P2P_FORMS:
        rs = [r for r in sweep if r.get("topology") == "ring" and r.get("form") == form and "ms" in r]
        ok = [r for r in rs if r.get("check") == "ok"]
        if not ok:
            continue
        b = min(ok, key=lambda r: r["ms"])
        alg = bucket / (b["ms"] * 1e-3) / 1e9
        out[form] = {"form_label": form_label("ring", form), "chunk_bytes": b["chunk_bytes"], "ms": b["ms"],
                     "pieces_swept": sorted({r["chunk_bytes"] for r in rs}),
                     "busbw_GBps_per_rank": round(alg * 2 * (world - 1) / world if world > 1 else alg, 2),
                     "roofline": allreduce_roofline(world, gpus, bucket, b["ms"], links_of(b)),
                     "judged": form == "direct"}
    return out or None


# The N > 1 line's stages after the default configuration, in the order they run: what the
# line must carry first -- the ring and default-topology RCCL entries (c4_ring), the bounded xGMI probe and
# the model's fit, C5 per width, the host-memory rate -- then the rest of the sweep, the model's refit and the
# re-timed headline; the extras last.  (name, required, reserve_s): a required stage always runs; an optional
# one runs only while the time left after it still covers every later required stage's reserve, and a
# bounded stage (the sweeps, the probe) gets exactly that much time.  Reserves are generous for a node (the
# loopback rehearsal's stages took 0.3-7 s each, its probe 40 s on one shared GPU).
DIST_STAGES = [
    ("sweep core", True, 30.0),
    ("xgmi probe", False, 10.0),
    ("C5 bf16", True, 40.0),
    ("host e2e", True, 30.0),
    ("sweep rest", False, 5.0),
    ("cost model", True, 5.0),
    ("headline", True, 15.0),
    ("phase timing", False, 8.0),
    ("rccl yardstick", False, 8.0),
    ("256 MiB", False, 8.0),
    ("reference cpu/mpi", False, 40.0),
]


class StageClock:
    """Time accounting of DIST_STAGES against the run's budget (FTAR_BENCH_BUDGET_S, which the watchdog
    enforces): `margin` seconds are kept for printing the line; the reserves, sized for the default 300 s, shrink
    with a smaller budget (a rehearsal's 100 s keeps every stage)."""

    def __init__(self, budget, t0, now=time.time, stages=DIST_STAGES, margin=10.0, budget_ref=300.0):
        self.budget, self.t0, self.now, self.margin = budget, t0, now, margin
        f = min(1.0, budget / budget_ref)
        self.stages = [(n, req, r * f) for n, req, r in stages]
        self.names = [st[0] for st in self.stages]
        self.skipped = {}

    def left(self):
        return self.budget - (self.now() - self.t0) - self.margin

    def reserved_after(self, name):
        i = self.names.index(name)
        return sum(r for _, req, r in self.stages[i + 1:] if req)

    def limit(self, name):
        """seconds this stage may take and still leave every later required stage its reserve"""
        return self.left() - self.reserved_after(name)

    def may_run(self, name):
        _, req, reserve = self.stages[self.names.index(name)]
        if req:
            return True
        ok = self.limit(name) >= reserve
        if not ok:
            self.skipped[name] = round(self.limit(name), 1)
        return ok


def run_stage_plan(clock, work):
    """Run DIST_STAGES with `work` = {name: fn(limit_s)} under `clock`: the order and the skipping rule of
    bench_distributed, kept apart so tests/test_bench_helpers.py can drive it with synthetic stage times.
    Returns the names run, in order."""
    ran = []
    for name in clock.names:
        if name not in work or not clock.may_run(name):
            continue
        work[name](clock.limit(name))
        ran.append(name)
    return ran


def sweep_form(form):
    """A sweep entry's form as the execution model prices it: (form name, registered) -- tuning suffixes
    (":ncclreg", ":plain", ":vec", ":dma", ":wgN") move the same bytes and are priced as their base
    form; "-reg" marks the peer forms on registered buffers (no local pass)."""
    base = form.split(":")[0]
    return (base[:-4], True) if base.endswith("-reg") else (base, False)


def predict_ms(ftar, topology, form, chunk, world, bucket):
    """The execution model's predicted ms for one sweep entry under the constants set now; None where it
    cannot price it (an unmeasured rate)."""
    name, reg = sweep_form(form)
    if name not in ftar.FORM:
        return None
    v = ftar.cost_predict("1" if topology == "ring" else topology, name, chunk, world, bucket, reg)
    return None if v is None else round(v * 1e3, 4)


def pieces_per_round(chunk, world, bucket, esz):
    """Pipeline pieces per round of one block (the engine's rule: chunk rounded down to 64 elements;
    0 = whole blocks)."""
    split = -(-(bucket // esz) // world)
    if not chunk:
        return 1
    c = max(64, (chunk // esz) & ~63)
    return max(1, -(-split // c))


def issue_from_enqueue(sweep, world, bucket, esz):
    """The host's enqueue time of one piece of one round (us): the median over the sweep's one-round RCCL
    entries of the time ftar_allreduce took to return (`enqueue_ms`) divided by the groups it issued
    (2 rounds x pieces).  Entries whose enqueue took at least half the call are left out: there RCCL's
    enqueue waited for the device (its work queue was full, so ncclGroupEnd blocks until earlier groups
    drain), which measures the device, not the host.  None without usable entries."""
    per = []
    for r in sweep:
        if (r.get("form") == "direct" and r.get("enqueue_ms") and r.get("check") == "ok" and
                r["enqueue_ms"] < 0.5 * r.get("ms", 0)):
            groups = 2 * pieces_per_round(r["chunk_bytes"], world, bucket, esz)
            per.append(r["enqueue_ms"] * 1e3 / groups)
    if not per:
        return None
    per.sort()
    return per[len(per) // 2]


# A fitted constant is reported "unidentified" (and the prior kept: the probe's value, or the default) when
# the sweep cannot pin it: fewer entries than free constants + 2, a value on its search bound, a flat
# direction -- doubling or halving it changes the summed squared log error by less than FLAT_SSE per entry
# (about a 1 % prediction change on average) -- or a ridge: held at 4x or 1/4 of its value, the OTHER
# constants re-fitted explain the sweep as well ("confounded", e.g. alpha and issue when every piece costs
# the same whichever term pays for it).  An ill-posed fit never sets the engine's constants.
FLAT_SSE = 1e-4


def _log_sse(ftar, pts, world, bucket):
    """summed squared log error of the model's predictions over `pts` under the constants set now"""
    import math
    e = 0.0
    for r in pts:
        p = predict_ms(ftar, r["topology"], r["form"], r["chunk_bytes"], world, bucket)
        if p is None or p <= 0:
            return float("inf")
        e += math.log(p / r["ms"]) ** 2
    return e


def _fit_log(f, x0, lo, hi, grid):
    """minimise f over a box in log space: the grid's best point (grid[d]: candidate values of coordinate
    d), then a pattern search from it (a step that improves is taken; none improving halves the steps, down
    to 1 %).  Returns (x, f(x))."""
    import itertools
    import math
    best = (float("inf"), list(x0))
    for y in itertools.product(*grid):
        fy = f(list(y))
        if fy < best[0]:
            best = (fy, list(y))
    x, fx = best[1], best[0]
    steps = [math.log(2.5) if len(g) > 1 else 0.0 for g in grid]
    while max(steps, default=0.0) > math.log(1.01):
        moved = False
        for d in range(len(x)):
            for sgn in (1, -1):
                if not steps[d]:
                    continue
                y = list(x)
                y[d] = min(hi[d], max(lo[d], x[d] * math.exp(sgn * steps[d])))
                fy = f(y)
                if fy < fx:
                    x, fx, moved = y, fy, True
                    break
        if not moved:
            steps = [s_ / 2 for s_ in steps]
    return x, fx


def _identify(f, x, fx, lo, hi, n, grid=None):
    """why each coordinate of the minimum x of f is not identified (None: it is): 'bound' (within 1 % of
    lo / hi), 'flat' (doubling and halving it both leave f within FLAT_SSE per entry) or, given the other
    coordinates' search grids, 'confounded' (held at 4x or 1/4 of its value, the others re-fitted reach f
    within FLAT_SSE per entry)"""
    why = []
    for d in range(len(x)):
        if x[d] <= lo[d] * 1.01 or x[d] >= hi[d] / 1.01:
            why.append("bound")
            continue
        moved = []
        for fac in (2.0, 0.5):
            y = list(x)
            y[d] = min(hi[d], max(lo[d], x[d] * fac))
            moved.append(f(y))
        if min(moved) - fx < FLAT_SSE * n:
            why.append("flat")
            continue
        conf = False
        for fac in ((4.0, 0.25) if grid and len(x) > 1 else ()):
            held = min(hi[d], max(lo[d], x[d] * fac))
            others = [i for i in range(len(x)) if i != d]

            def g(z):
                y = list(x)
                y[d] = held
                for i, v in zip(others, z):
                    y[i] = v
                return f(y)
            _, fz = _fit_log(g, [x[i] for i in others], [lo[i] for i in others], [hi[i] for i in others],
                             [grid[i] for i in others])
            conf = conf or fz - fx < FLAT_SSE * n
        why.append("confounded" if conf else None)
    return why


def refit_cost_model(ftar, sweep, world, bucket, fixed=None):
    """The execution model's p2p constants re-fitted to this run's own sweep: alpha (one p2p
    group), link (one peer, one direction) and issue (host enqueue of one piece) minimise the squared log
    error of the model's prediction over the validated RCCL p2p entries (forms direct / stages, no tuning
    suffix; several topologies and piece sizes): a log grid, then a pattern search.  `fixed` names constants
    measured directly (e.g. {"issue_us": ...}) that the search keeps.  A constant the sweep cannot pin
    (fewer entries than free constants + 2, a search bound, a flat direction) keeps its prior -- the value
    set when the refit started (the probe's, or the default) -- and is listed in "unidentified" with the
    reason; the others are fitted again with it held, and if the result predicts the sweep no better than
    the prior constants did, the priors are kept whole ("kept_prior").  Leaves the model on the result and
    returns {"params", "entries", "rms_log_err", "rms_log_err_prior", "unidentified", "prior",
    "kept_prior"} (None: no validated entry)."""
    import math
    pts = [r for r in sweep if r.get("check") == "ok" and "ms" in r and r.get("form") in ("direct", "stages")]
    if not pts:
        return None
    base = ftar.cost_get()
    fixed = {k: v for k, v in (fixed or {}).items() if v}
    names = ["alpha_us", "link_gbps", "issue_us"]
    lo_all = {"alpha_us": 0.1, "link_gbps": 0.5, "issue_us": 0.1}          # us, GB/s, us
    hi_all = {"alpha_us": 1e5, "link_gbps": 5e3, "issue_us": 1e5}
    grid_all = {"alpha_us": (0.5, 5000.0, 11), "link_gbps": (1.0, 1000.0, 13), "issue_us": (0.5, 5000.0, 11)}
    unidentified = {}

    def geom(lo, hi, n):
        return [lo * (hi / lo) ** (i / (n - 1)) for i in range(n)]

    def solve(free):
        held = dict(fixed, **{k: base[k] for k in unidentified})

        def f(y):
            ftar.cost_set(**dict(base, **held, **dict(zip(free, y))))
            return _log_sse(ftar, pts, world, bucket)
        x, fx = _fit_log(f, [base[k] for k in free], [lo_all[k] for k in free], [hi_all[k] for k in free],
                         [geom(*grid_all[k]) for k in free])
        return f, x, fx, [geom(lo_, hi_, 7) for lo_, hi_, _ in (grid_all[k] for k in free)]

    free = [k for k in names if k not in fixed]
    if len(pts) < len(free) + 2:
        unidentified.update({k: f"entries ({len(pts)} < {len(free)} free + 2)" for k in free})
        free = []
    for _ in range(len(names)):          # drop what the sweep cannot pin, fit the rest again
        if not free:
            break
        f, x, fx, coarse = solve(free)
        why = _identify(f, x, fx, [lo_all[k] for k in free], [hi_all[k] for k in free], len(pts), coarse)
        bad = {k: w for k, w in zip(free, why) if w}
        if not bad:
            break
        unidentified.update(bad)
        free = [k for k in free if k not in bad]
    final = dict(base, **fixed, **{k: base[k] for k in unidentified})
    if free:
        final.update(dict(zip(free, x)))
    ftar.cost_set(**dict(base, **fixed))
    sse_prior = _log_sse(ftar, pts, world, bucket)
    params = ftar.cost_set(**final)
    sse = _log_sse(ftar, pts, world, bucket)
    kept_prior = bool(free) and not sse < sse_prior
    if kept_prior:   # the fit explains the sweep no better than the constants it started from: keep those
        params = ftar.cost_set(**dict(base, **fixed))
        sse = sse_prior

    def rms(e):
        return round(math.sqrt(e / len(pts)), 4) if e < float("inf") else None
    return {"params": {k: round(v, 3) for k, v in params.items()}, "entries": len(pts), "rms_log_err": rms(sse),
            "rms_log_err_prior": rms(sse_prior), "unidentified": unidentified,
            "prior": {k: round(base[k], 3) for k in unidentified},
            "kept_prior": "the refit predicted the sweep no better than the prior constants" if kept_prior else None}


def refit_form_rate(ftar, sweep, world, bucket, field, forms):
    """One more constant of the execution model fitted to this run's sweep: the rate `field` (peer_read_gbps,
    peer_write_gbps or coll_gbps) that minimises the squared log error over the validated entries whose form
    is in `forms` (a 1-D golden-section search in log space, 1 .. 5000 GB/s).  Unidentified (fewer than 3
    entries, a search bound, a flat direction): the prior -- the value set when the refit started, the
    probe's or the default -- is kept and the reason given.  Leaves the model on the result; returns
    {"value", "entries", "rms_log_err", "unidentified"} or None (no entries)."""
    import math
    pts = [r for r in sweep if r.get("check") == "ok" and "ms" in r and r.get("form") in forms]
    if not pts:
        return None
    base = ftar.cost_get()
    lo, hi = 1.0, 5000.0

    def err_at(v):
        ftar.cost_set(**dict(base, **{field: v}))
        return _log_sse(ftar, pts, world, bucket)

    def rms(e):
        return round(math.sqrt(e / len(pts)), 4) if e < float("inf") else None
    if len(pts) < 3:
        ftar.cost_set(**base)
        return {"value": round(base[field], 3), "entries": len(pts), "unidentified": f"entries ({len(pts)} < 3)",
                "rms_log_err": rms(_log_sse(ftar, pts, world, bucket))}
    a, b = math.log(lo), math.log(hi)
    g = (math.sqrt(5) - 1) / 2
    c, d = b - g * (b - a), a + g * (b - a)
    fc, fd = err_at(math.exp(c)), err_at(math.exp(d))
    while b - a > 1e-3:
        if fc < fd:
            b, d, fd = d, c, fc
            c = b - g * (b - a)
            fc = err_at(math.exp(c))
        else:
            a, c, fc = c, d, fd
            d = a + g * (b - a)
            fd = err_at(math.exp(d))
    v = math.exp((a + b) / 2)
    e = err_at(v)
    why = _identify(lambda y: err_at(y[0]), [v], e, [lo], [hi], len(pts))[0]
    if why:
        ftar.cost_set(**base)
        return {"value": round(base[field], 3), "entries": len(pts), "unidentified": why,
                "fitted_at": round(v, 3), "rms_log_err": rms(_log_sse(ftar, pts, world, bucket))}
    err_at(v)
    return {"value": round(v, 3), "entries": len(pts), "rms_log_err": rms(e), "unidentified": None}


def _factorizations(n):
    out = []

    def rec(m, cur):
        if m == 1:
            if cur:
                out.append(list(cur))
            return
        for f in range(2, m + 1):
            if m % f == 0:
                rec(m // f, cur + [f])
    rec(n, [])
    return out


def bench_distributed(a):
    """N > 1: one rank per GPU.  Order of work, safest first, so that a configuration that hangs on a node
    cannot cost the run its result:
      1. the default configuration (FT_TOPO/--topo, else the cost model; RCCL p2p, direct forms) timed for
         exactly K steps after W warmup -- the headline unless the sweep finds a faster *validated* one;
      2. the sweep (BASELINE configs[3]: topology x chunk x data-movement form) inside a time budget every
         rank agrees on, in tiers: the default topology's direct RCCL forms, its IPC peer forms (after the
         xGMI probe), the other topologies' direct/collective forms, the staged rounds, other peer forms;
      3. the sweep's best, re-timed for exactly K steps after W warmup, if it beats the default;
      4. RCCL's own ncclAllReduce on the same bucket (yardstick).
    A watchdog (FTAR_BENCH_BUDGET_S, default 300 s) prints the best line measured so far and ends every
    rank if anything hangs."""
    import threading

    import torch
    import torch.distributed as dist

    import ftar
    import ftar.dist

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    t_start = time.time()
    budget = float(os.environ.get("FTAR_BENCH_BUDGET_S", "300"))
    sweep_budget = float(os.environ.get("FTAR_BENCH_SWEEP_S", "150"))
    state = {"line": None, "printed": False, "done": False, "phase": "init", "major": ("init", t_start)}
    lock = threading.Lock()

    def emit(res):
        with lock:
            if rank == 0 and not state["printed"]:
                print(json.dumps(res), flush=True)
            state["printed"] = True

    def watchdog():
        while time.time() - t_start < budget:
            time.sleep(1.0)
            if state["done"]:
                return
        sys.stderr.write(f"[bench rank {rank}] watchdog: {budget:.0f}s exceeded in phase {state['phase']}\n")
        import faulthandler
        faulthandler.dump_traceback(file=sys.stderr, all_threads=True)   # where every thread of this rank is
        cut = dict(stage_t, **({state["major"][0] + " (cut)": round(time.time() - state["major"][1], 2)}
                                if state.get("major") else {}))
        if state["line"] is not None:
            res = dict(state["line"])
            res["watchdog"] = f"run cut at {budget:.0f}s in phase '{state['phase']}'; headline = last complete measurement"
            res["stage_wall_s"] = cut
            emit(res)
        else:   # nothing measured yet: still one line, saying where every stage's time went
            emit({"metric": "fp32 bucket reduce-sum GB/s (device-resident) at 1/2/4/8 MI355X", "value": None,
                  "unit": "GB/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": None,
                  "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": a.dtype,
                  "data": "synthetic", "config": {"workload": f"{world}xMI355X FlexTree AllReduce over xGMI"},
                  "watchdog": f"run cut at {budget:.0f}s in phase '{state['phase']}' before any measurement",
                  "stage_wall_s": cut, "rccl_error_by_rank": state.get("rccl_ranks")})
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0 if state["line"] is not None else 3)

    threading.Thread(target=watchdog, daemon=True).start()

    stage_t = {}   # major stage -> wall seconds (this rank), reported as stage_wall_s

    def phase(name, major=True):
        """progress on stderr (rank 0): a long N>1 run never looks idle; major stages are timed"""
        now = time.time()
        if major:
            last = state.get("major")
            if last is not None:
                stage_t[last[0]] = round(stage_t.get(last[0], 0.0) + now - last[1], 2)
            state["major"] = (name, now)
        state["phase"] = name
        if rank == 0:
            sys.stderr.write(f"[bench {time.time() - t_start:7.1f}s] {name}\n")
            sys.stderr.flush()

    dist.init_process_group("gloo")   # host-side barrier/max only; the data path is ftar+RCCL

    def all_errors(err):
        """every rank's view of a failure (its exception and ftar_last_error), gathered over gloo, so one
        driver record diagnoses a first RCCL contact that failed on some rank"""
        mine = {"rank": rank, "error": err or "", "ftar_last_error": ftar.last_error()}
        allv = [None] * world
        dist.all_gather_object(allv, mine)
        return allv
    if a.host_comm or world > torch.cuda.device_count():
        # rehearsal: ranks share the visible GPUs, IPC peer forms over a gloo-bootstrapped communicator;
        # exercises this whole function at P > 1 on a 1-GPU box (timings are not xGMI numbers).  Without
        # --host-comm RCCL refuses the shared GPU and the run takes the fallback below.
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    comm, rccl_error, rccl_ranks = None, None, None
    if a.rccl_loopback and not a.host_comm:
        # one "host" per rank for RCCL: its duplicate-GPU check compares (host hash, bus id), and ranks on
        # different hosts talk through the network transport (sockets on lo), never IPC or xGMI
        os.environ["NCCL_HOSTID"] = f"ftar-loopback-{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
        if rank == 0 and world <= torch.cuda.device_count():
            sys.stderr.write("[bench] --rccl-loopback with a GPU per rank: RCCL moves the data over sockets, "
                             "not xGMI; drop the flag to measure the node\n")
    if not a.host_comm:
        try:
            comm = ftar.dist.init_comm(device=local)   # RCCL unique id over the gloo group
        except Exception as e:  # noqa: BLE001
            rccl_error = str(e)[:200]
        ok = torch.tensor([0 if rccl_error else 1], dtype=torch.int32)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)   # every rank takes the same path
        if not ok.item():
            rccl_ranks = all_errors(rccl_error)
            state["rccl_ranks"] = rccl_ranks
            # RCCL could not come up on some rank: the peer forms over a gloo-bootstrapped communicator still
            # move the data over xGMI (IPC), so the run keeps a measured line
            if comm is not None:
                comm.destroy()
                comm = None
            sys.stderr.write(f"[bench rank {rank}] RCCL communicator failed ({rccl_error or 'on another rank'}); "
                             "falling back to the host-bootstrapped peer forms\n")
            a.host_comm = True
    if comm is None:
        comm = ftar.dist.init_host_comm(device=local)
    # the default configuration's data movement: the execution model's choice per call ("auto"); a
    # host-bootstrapped communicator moves data by the peer forms only
    base_form = "peer-read" if a.host_comm else "auto"
    n = a.n or (1 << 28)
    esz = ftar.dtype_size(a.dtype)
    tdt = {"f32": torch.float32, "bf16": torch.bfloat16}[a.dtype]
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + rank)
    x = (torch.rand(n, generator=gen, device=dev, dtype=torch.float32) * 2 - 1).to(tdt)
    y = torch.empty_like(x)
    stream = torch.cuda.current_stream()
    bucket = n * esz
    # after an RCCL call that never completed (preflight below), a device-wide synchronize would wait on it
    # forever: from then on only the bench stream is synchronised (every ftar call joins it at its end)
    sync_state = {"device": True}

    def sync():
        if sync_state["device"]:
            torch.cuda.synchronize()
        else:
            stream.synchronize()

    def preflight(timeout_s):
        """First contact of RCCL p2p between the ranks: one small call of the default configuration, waited
        for with a deadline, so a transfer that never completes becomes the IPC fallback below instead of a
        run the watchdog cuts with nothing measured.  The call itself is bounded too: its first contact (the
        settings all-gather and RCCL's p2p connections, which block the host) runs under
        FTAR_FIRST_CONTACT_TIMEOUT_S = timeout_s and fails with FTAR_ERR_TIMEOUT instead of hanging
        (ADVICE r3).  FTAR_BENCH_PREFLIGHT_HANG=1 rehearses the path with a stream that really does not drain
        (a spinning wave, libftar_bench.so, released at the end of the run).  Returns "" or why not."""
        npf = min(n, 1 << 20)
        os.environ["FTAR_FIRST_CONTACT_TIMEOUT_S"] = str(timeout_s)
        try:
            comm.chunk_bytes = default_chunk
            comm.peer_direct, comm.allgather, comm.reduce_scatter = 0, "direct", "direct"
            try:
                comm.allreduce(x[:npf], y[:npf], npf, a.dtype, "sum", topo_=default_topo, stream=stream)
            except ftar.FtarError as e:
                if e.status == 7:   # FTAR_ERR_TIMEOUT: the first contact never completed
                    return f"RCCL preflight ({npf} elements) not complete after {timeout_s:.0f}s: {str(e)[:160]}"
                raise
            if os.environ.get("FTAR_BENCH_PREFLIGHT_HANG"):   # rehearsal: this stream now really never drains
                import ctypes
                lib = ftar.bench_lib()
                lib.ftar_debug_block_stream.restype = ctypes.c_void_p
                lib.ftar_debug_block_stream.argtypes = [ctypes.c_void_p, ctypes.c_double]
                # the wave spins until released at the end of the run, or this limit: past the fallback's
                # default measurement, which must still find the stream blocked
                state["blocked_flag"] = lib.ftar_debug_block_stream(stream.cuda_stream, 3 * timeout_s + 10)
            ev = torch.cuda.Event()
            ev.record(stream)
            state["preflight_ev"] = ev
            t_end = time.time() + timeout_s
            while not ev.query():
                if time.time() > t_end:
                    return f"RCCL preflight ({npf} elements) not complete after {timeout_s:.0f}s"
                time.sleep(0.005)
            return ""
        except Exception as e:  # noqa: BLE001
            return f"RCCL preflight failed: {str(e)[:180]}"

    def unblock():
        """the rehearsal's spinning wave (FTAR_BENCH_PREFLIGHT_HANG), released so the device drains"""
        if state.get("blocked_flag"):
            import ctypes
            lib = ftar.bench_lib()
            lib.ftar_debug_unblock.argtypes = [ctypes.c_void_p]
            lib.ftar_debug_unblock(state.pop("blocked_flag"))

    enq = {"ms": None}   # the last timed() run's host enqueue time per call (median, max over ranks)

    def timed(fn, steps, warmup):
        """barrier + sync on both sides of `steps` calls; max over ranks (ms per call).  Also the host time
        each call took to return (ftar_allreduce returns once everything is enqueued): its median, max over
        ranks, in enq["ms"] -- the enqueue cost the execution model's `issue` constant prices."""
        for _ in range(warmup):
            fn()
        sync()
        dist.barrier()
        sync()
        per = []
        t0 = time.perf_counter()
        for _ in range(steps):
            t1 = time.perf_counter()
            fn()
            per.append(time.perf_counter() - t1)
        sync()
        dist.barrier()
        per.sort()
        t = torch.tensor([time.perf_counter() - t0, per[len(per) // 2] if per else 0.0], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        enq["ms"] = round(t[1].item() * 1e3, 4)
        return t[0].item() / max(1, steps) * 1e3

    def run_with(topo, chunk, form="direct"):
        """form: "direct" (one-round reduce-scatter and all-gather over RCCL p2p), "stages" (the reference's
        rounds both ways), "collective" (ncclAllGather), "peer-read" / "peer-write" (one-round plan moved by
        kernel loads / stores through IPC-mapped exchange buffers), "...-reg" (the same on registered buffers,
        no local pass), "auto" (the execution model's form per call, and its piece where chunk is 0; the
        topology is `topo`, or the model's too when topo is None)."""
        # peer-form tuning suffix: ":plain" = plain (not nontemporal) copies, ":vec" = register-kernel fold,
        # ":dma" = the cross-GPU copies by the DMA engines
        form, _, tune = form.partition(":")
        comm.peer_tuning(nt=tune != "plain", lds=tune != "vec", dma=tune == "dma")
        # (no ":cusN": a CU-masked reduce stream is refused on RCCL communicators)
        # ":ncclreg": RCCL p2p between buffers registered with RCCL (ncclCommRegister): the comm's scratch
        # and registered copies of x and y, so RCCL may skip its staging copies where it supports that
        comm.rccl_register = tune == "ncclreg"
        # ":wgN": the peer forms' cross-GPU copies capped at N workgroups per segment (the probe's best cap)
        comm.peer_wg_cap = int(tune[2:]) if tune.startswith("wg") else 0
        comm.chunk_bytes = chunk
        if form == "auto":
            comm.form = "auto"
        else:
            peer = form.startswith("peer-")
            comm.peer_direct = form.split("-")[1] if peer else 0
            comm.allgather = "direct" if peer else form
            comm.reduce_scatter = "stages" if form == "stages" else "direct"
        xin, yout = (reg_bufs() if form.endswith("-reg") or tune == "ncclreg" else (x, y))

        def fn():
            comm.allreduce(xin, yout, n, a.dtype, "sum", topo_=topo, stream=stream)
        fn.xin, fn.yout = xin, yout
        return fn

    reg = {}

    def reg_bufs():
        """x and y copies registered with the communicator (ftar_comm_register, collective, once): the peer
        forms then read / write the peers' buffers in place, with no local pass."""
        if not reg:
            reg["x"], reg["y"] = x.clone(), torch.empty_like(y)
            sync()
            reg["ids"] = [comm.register(reg["x"], bucket), comm.register(reg["y"], bucket)]
        return reg["x"], reg["y"]

    def fit_cost_model(probe):
        """The execution model's constants from this node's probe, before the sweep prices
        anything: link = the probe's per-link, per-direction copy rate; peer read / write = the probe's
        read / write from all peers per link (so the peer forms become candidates); alpha = half a 4 KiB
        direct-form AllReduce (two p2p rounds, no bandwidth term to speak of); barrier = a third of a 4 KiB
        peer-read call (three barriers).  Set process-wide on every rank alike (rank 0's values broadcast),
        so every later choice uses them; the sweep then re-fits the p2p constants to its own timings."""
        default = ftar.cost_get()
        link = link_rate_from_probe(probe, world)

        def per_link(key):
            v = (probe or {}).get(key)
            v = v[0] if isinstance(v, (list, tuple)) else v
            return v / max(1, world - 1) if isinstance(v, (int, float)) and v > 0 else 0.0
        small = torch.zeros(1024, device=dev)
        small_y = torch.empty_like(small)
        comm.peer_tuning()
        comm.chunk_bytes = 0
        comm.peer_direct = "read" if base_form.startswith("peer-") else 0   # host-bootstrapped: peer forms only
        comm.allgather, comm.reduce_scatter = "direct", "direct"
        t_small = ftar.topo(str(world))
        ms_small = timed(lambda: comm.allreduce(small, small_y, 1024, "f32", "sum", topo_=t_small, stream=stream),
                         20, 3)
        comm.peer_direct = "read"
        ms_peer = timed(lambda: comm.allreduce(small, small_y, 1024, "f32", "sum", topo_=t_small, stream=stream),
                        20, 3)
        v = torch.tensor([link or 0.0, ms_small, ms_peer, per_link("read_all_peers"), per_link("write_all_peers")],
                         dtype=torch.float64)
        dist.broadcast(v, 0)  # one set of constants on every rank: identical choices everywhere
        link, ms_small, ms_peer, pr, pw = (x.item() for x in v)
        fitted = ftar.cost_set(**dict(default, alpha_us=ms_small * 1e3 / 2, link_gbps=link or 0.0,
                                      barrier_us=ms_peer * 1e3 / 3, peer_read_gbps=pr, peer_write_gbps=pw))
        t_ref, _ = ftar.topo_choose_reference(world)
        return {"default": {k: round(x, 3) for k, x in default.items()},
                "fitted": {k: round(x, 3) for k, x in fitted.items()},
                "source": "link, peer read/write: ftar_xgmi_probe per-link one-direction rates (rank 0); alpha: "
                          "half a 4 KiB direct AllReduce; barrier: a third of a 4 KiB peer-read call"
                          + ("" if link else "; probe gave no link rate: default link kept"),
                "choice_fitted": ftar.exec_choose(world, bucket).as_dict(),
                "choice_reference_model": str(t_ref)}

    def validate_model(sweep):
        import math
        keys = list(ftar.cost_get())
        before = ftar.cost_get()
        for r in sweep:
            if "ms" in r:
                r["model_ms"] = predict_ms(ftar, r["topology"], r["form"], r["chunk_bytes"], world, bucket)

        def log_err(field):
            e = [abs(math.log(r[field] / r["ms"])) for r in sweep
                 if r.get("check") == "ok" and r.get(field) and r.get("ms")]
            e.sort()
            return {"median_abs_log_err": round(e[len(e) // 2], 4) if e else None, "entries": len(e)}
        issue = issue_from_enqueue(sweep, world, bucket, esz)
        p2p = refit_cost_model(ftar, sweep, world, bucket, fixed={"issue_us": issue} if issue else None)
        rates = {f: refit_form_rate(ftar, sweep, world, bucket, f, forms)
                 for f, forms in (("peer_read_gbps", ("peer-read", "peer-read-reg")),
                                  ("peer_write_gbps", ("peer-write", "peer-write-reg")),
                                  ("coll_gbps", ("collective",)))}
        v = torch.tensor([ftar.cost_get()[k] for k in keys], dtype=torch.float64)
        dist.broadcast(v, 0)   # one set of constants on every rank: identical choices everywhere
        refit = ftar.cost_set(**dict(zip(keys, v.tolist())))
        for r in sweep:
            if "ms" in r:
                r["model_ms_refit"] = predict_ms(ftar, r["topology"], r["form"], r["chunk_bytes"], world, bucket)
        ok = [r for r in sweep if r.get("check") == "ok" and "ms" in r]
        best = min(ok, key=lambda r: r["ms"]) if ok else None
        fixed = default_topo if (a.topo or os.environ.get("FT_TOPO")) else None
        if a.host_comm:   # no p2p transfers: the model chooses between the peer forms only
            cands = []
            for f in ("peer-read", "peer-write"):
                try:
                    cands.append(ftar.exec_choose(world, bucket, topo_=fixed or default_topo, form=f, chunk_bytes=0))
                except ftar.FtarError:   # that form's rate is unmeasured (the probe did not run)
                    pass
            if not cands:
                return {"constants_probe": before, "note": "no peer-form rate measured: nothing to choose"}
            ch = min(cands, key=lambda c: c.seconds).as_dict()
        else:
            ch = ftar.exec_choose(world, bucket, topo_=fixed, chunk_bytes=a.chunk_bytes or None,
                                  peer=True).as_dict()
        ch_chunk = ch["chunk_bytes"] or -(-n // world) * esz
        same = [r for r in ok if r["topology"] == ch["topology"] and r["form"] == ch["form"] and
                pieces_per_round(r["chunk_bytes"], world, bucket, esz) ==
                pieces_per_round(ch_chunk, world, bucket, esz)]
        if same:
            measured = min(r["ms"] for r in same)
        else:   # not in the sweep: time it (validated like every entry)
            fn = run_with(ftar.topo("1" if ch["topology"] == "ring" else ch["topology"]),
                          0 if ch["form"].startswith("peer") else ch_chunk, ch["form"])
            measured = timed(fn, steps=min(5, a.steps), warmup=1)
            okc, whyc = check_y(fn)
            sweep.append({"topology": ch["topology"], "chunk_bytes": ch_chunk, "form": ch["form"],
                          "ms": round(measured, 4), "busbw_GBps": round(bws(measured)[1], 2), "enqueue_ms": enq["ms"],
                          "check": "ok" if okc else f"MISMATCH ({whyc})", "source": "the refit model's choice",
                          "model_ms_refit": round(ch["predicted_ms"], 4)})
            if not okc:
                measured = None
        return {"constants_probe": {k: round(x, 3) for k, x in before.items()},
                "constants_refit": {k: round(x, 3) for k, x in refit.items()},
                "refit_p2p": p2p, "refit_rates": rates, "issue_us_from_enqueue": issue,
                "prediction_error_probe": log_err("model_ms"), "prediction_error_refit": log_err("model_ms_refit"),
                "choice_refit": ch, "choice_refit_measured_ms": None if measured is None else round(measured, 4),
                "sweep_best": None if best is None else {k: best[k] for k in ("topology", "form", "chunk_bytes", "ms")},
                "regret_refit": None if (measured is None or best is None) else round(measured / best["ms"] - 1, 4),
                "note": "model_ms (per sweep entry): the prediction under the probe-fitted constants; model_ms_refit: "
                        "under the constants re-fitted to this sweep; regret = the refit choice's measured ms over "
                        "the sweep's best, minus 1"}

    # correctness of y: identical on every rank, and within (P-1) * eps * sum|x| of the fp64 sum on a sample
    idx = sample_index(n, dev)
    xs = x[idx].float().cpu()
    allx = [torch.empty_like(xs) for _ in range(world)]
    dist.all_gather(allx, xs)
    ref64 = sum(t.double() for t in allx)
    absum = sum(t.double().abs() for t in allx)
    eps = 2.0 ** -24 if a.dtype == "f32" else 2.0 ** -8
    tol = (world - 1) * eps * absum + 1e-30

    def check_y(fn):
        """y (from the timed calls) against the fp64 sample and across ranks; then one more call on the
        negated inputs must give exactly -y everywhere (round-to-nearest-even is sign-symmetric), which
        proves the call read this call's data (no stale copies) over the whole bucket.  Returns (ok, what
        failed on any rank: "" | "sample" | "ranks differ" | "negation")."""
        x, y = fn.xin, fn.yout
        sync()
        mine = y[idx].float().cpu()
        ally = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(ally, mine)
        bits = 0
        if not all(torch.equal(ally[0], t) for t in ally):
            bits |= 2
        if not bool(((mine.double() - ref64).abs() <= tol).all()):
            bits |= 1
        y1 = y.clone()
        x.neg_()
        try:
            fn()
            sync()
        finally:
            x.neg_()   # the inputs stay intact for the next configuration, whatever happened
        if not torch.equal(y, y1.neg_()):
            bits |= 4
        del y1
        allb = [torch.zeros(1, dtype=torch.int32) for _ in range(world)]   # every rank's failures, OR-ed
        dist.all_gather(allb, torch.tensor([bits], dtype=torch.int32))
        bits = 0
        for b in allb:
            bits |= int(b.item())
        why = ", ".join(w for bit, w in ((1, "sample"), (2, "ranks differ"), (4, "negation")) if bits & bit)
        return bits == 0, why

    def measure_c5():
        """BASELINE configs[4]: the bf16 1 GiB bucket with the cost model's width -- topology, form and piece
        all the execution model's (FT_TOPO / --topo fix the topology), then every other width the model
        weighed, each with the form and piece the model gives it, timed against its prediction."""
        nb = a.n_c5 or (1 << 29)
        xb = (torch.rand(nb, generator=gen, device=dev, dtype=torch.float32) * 2 - 1).to(torch.bfloat16)
        yb = torch.empty_like(xb)
        fixed = ftar.topo(a.topo, a.lonely, nranks=world) if a.topo else None   # None: FT_TOPO, else the model
        comm.chunk_bytes = a.chunk_bytes
        comm.rccl_register = False
        comm.peer_tuning()
        comm.reduce_cus = 0
        if a.host_comm:
            comm.peer_direct = "read"
        else:
            comm.form = "auto"

        def fn5():
            comm.allreduce(xb, yb, nb, "bf16", "sum", topo_=fixed, stream=stream)
        ms5 = timed(fn5, min(a.steps, 10), 2)
        chosen = comm.last_exec()
        t5 = ftar.topo("1" if chosen["topology"] == "ring" else chosen["topology"])
        # validation: every rank identical; within one bf16 rounding per fold level (at most P) of the fp64 sum
        ix = sample_index(nb, dev)
        xs5 = xb[ix].double().cpu()
        ax = [torch.empty_like(xs5) for _ in range(world)]
        dist.all_gather(ax, xs5)
        r64, ab = sum(ax), sum(t.abs() for t in ax)
        mine = yb[ix].double().cpu()
        ay = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(ay, mine)
        ok5 = all(torch.equal(ay[0], t) for t in ay) and bool(((mine - r64).abs() <= world * 2.0 ** -8 * ab + 1e-30).all())
        flag = torch.tensor([1 if ok5 else 0], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        alg5 = nb * 2 / (ms5 * 1e-3) / 1e9
        # the other widths the cost model weighed (every ordered factorization of P, and the ring), a few
        # timed calls each with the form and piece the model gives them: does its choice hold on this node?
        widths = {}
        for tp in ["1"] + [",".join(map(str, f)) for f in _factorizations(world)]:
            tw = ftar.topo(tp)
            if str(tw) == str(t5) or world < 2:
                continue
            try:
                mw = timed(lambda: comm.allreduce(xb, yb, nb, "bf16", "sum", topo_=tw, stream=stream), 3, 1)
                ex = comm.last_exec()
                widths[str(tw)] = {"ms": round(mw, 4), "form": ex["form"], "form_label": form_label(tw, ex["form"]),
                                   "chunk_bytes": ex["chunk_bytes"],
                                   "model_ms": None if ex["predicted_ms"] is None else round(ex["predicted_ms"], 4)}
            except Exception as e:  # noqa: BLE001
                widths[str(tw)] = {"error": str(e)[:120]}
        del xb, yb
        return {"workload": f"{world}xMI355X FlexTree AllReduce, bf16 2^{nb.bit_length() - 1} elements per rank "
                            "(BASELINE configs[4])", "topology": str(t5), "form": chosen["form"],
                "form_label": form_label(t5, chosen["form"]),
                # the width choice said out loud: in the direct form every one-round width prices alike, and the
                # model then keeps the fewest stages -- a tie, not a score
                "model_tied": chosen.get("tied"), "model_tie_broken_by": chosen.get("tie_broken_by"),
                "chunk_bytes": chosen["chunk_bytes"], "ms": round(ms5, 4), "value_GBps": round(world * alg5, 2),
                "algbw_GBps_per_rank": round(alg5, 2),
                "busbw_GBps_per_rank": round(alg5 * 2 * (world - 1) / world if world > 1 else alg5, 2),
                "check": "ok" if bool(flag.item()) else "MISMATCH",
                "model_ms": None if chosen["predicted_ms"] is None else round(chosen["predicted_ms"], 4),
                "selection": "FT_TOPO / --topo" if (fixed is not None or os.environ.get("FT_TOPO"))
                             else "the execution model (topology, form, piece)",
                "cost_model_params": ftar.cost_get(),
                "reference_model_choice": str(ftar.topo_choose_reference(world)[0]),
                "other_widths": widths}

    def measure_host():
        """The reference's setting: the bucket lives in host memory (MPI send/recv buffers,
        benchmark.cpp:125-131).  Pinned host buckets through ftar_allreduce_host -- H2D, the exchange and D2H
        pipelined per piece -- with the default topology; the same plan gives the device path's bits."""
        hx = x.cpu().pin_memory()
        hy = torch.empty_like(hx).pin_memory()
        comm.chunk_bytes = default_chunk
        # RCCL: the p2p host path; a host-bootstrapped communicator: the read form piece by piece
        comm.peer_direct = "read" if a.host_comm else 0
        comm.allgather = "direct"
        comm.reduce_scatter = "direct"
        comm.peer_tuning()
        comm.reduce_cus = 0   # the sweep's last configuration may have left the reduce stream on a CU subset
        comm.rccl_register = False

        def fnh():
            comm.allreduce_host(hx, hy, n, a.dtype, "sum", topo_=default_topo, stream=stream)
        msh = timed(fnh, min(a.steps, 5), 1)
        fn_default()   # the device path on the same inputs: y
        sync()
        ic = idx.cpu()
        same = torch.tensor([1 if torch.equal(hy[ic], y[idx].cpu()) else 0], dtype=torch.int32)
        dist.all_reduce(same, op=dist.ReduceOp.MIN)
        alg = bucket / (msh * 1e-3) / 1e9
        del hx, hy
        return {"workload": f"{world}xMI355X host-memory AllReduce (pinned buckets, H2D + exchange + D2H "
                            "pipelined; ftar_allreduce_host, the MPI_Allreduce_FT path)",
                "topology": str(default_topo), "ms": round(msh, 4), "value_GBps": round(world * alg, 2),
                "algbw_GBps_per_rank": round(alg, 2),
                "check": "bit-identical to the device path" if same.item() else "MISMATCH"}

    def bws(m):
        alg = bucket / (m * 1e-3) / 1e9
        return alg, (alg * 2 * (world - 1) / world if world > 1 else alg)

    def make_result(ms, topo_, chunk, form, ok, steps, warmup, extra):
        algbw, busbw = bws(ms)
        links = links_driven(world, str(topo_), form)
        probe = state.get("line", {}).get("xgmi_probe_GBps") if isinstance(state.get("line"), dict) else None
        roof = allreduce_roofline(world, torch.cuda.device_count(), bucket, ms, links,
                                  link_rate_from_probe(probe, world))
        res = {
            "metric": "fp32 bucket reduce-sum GB/s (device-resident) at 1/2/4/8 MI355X",
            "value": round(world * algbw, 2), "unit": "GB/s", "n_gpus": world, "steps": steps,
            "warmup": warmup, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": a.dtype, "data": "synthetic (torch.rand uniform [-1,1), HBM-resident)",
            "config": {"workload": f"{world}xMI355X FlexTree AllReduce over xGMI, "
                                   f"{'IPC-mapped' if form.startswith('peer-') else 'RCCL p2p'}, "
                                   f"{form_label(topo_, form)} (BASELINE configs[2-3])",
                       "bucket_bytes": bucket, "elements_per_rank": n, "topology": str(topo_),
                       "chunk_bytes": chunk, "form": form, "form_label": form_label(topo_, form),
                       "xgmi_links": links, "parallelism": f"dp{world}"
                       + (f" (rehearsal: {world} ranks on {torch.cuda.device_count()} GPU(s), host-bootstrapped "
                          "communicator; not an xGMI measurement)" if a.host_comm and world > torch.cuda.device_count()
                          else f" (rehearsal: {world} ranks on {torch.cuda.device_count()} GPU(s), RCCL over loopback "
                          "sockets, one NCCL_HOSTID per rank; not an xGMI measurement)"
                          if a.rccl_loopback and world > torch.cuda.device_count()
                          else " (host-bootstrapped communicator: RCCL unavailable, see rccl_init_error)" if a.host_comm else "")},
            "algbw_GBps_per_rank": round(algbw, 2), "busbw_GBps_per_rank": round(busbw, 2),
            "roofline": roof,
            "value_convention": "value = N x bucket bytes / t (aggregate algBW); algbw = bucket / t per rank; "
                                "busbw = algbw x 2(P-1)/P",
            "check": "ok" if ok else "MISMATCH",
        }
        if rccl_error:
            res["rccl_init_error"] = rccl_error
            res["rccl_error_by_rank"] = rccl_ranks
        res.update(extra)
        return res

    # 1. the default configuration: FT_TOPO/FT_LONELY (or --topo), else the re-fitted cost model
    phase("default")
    # the default configuration is the execution model's: FT_TOPO / --topo fix the topology,
    # --chunk-bytes the piece; the rest -- topology, form, piece -- comes from the model under its default
    # constants (no rate of this node is known yet, so the peer forms are not candidates)
    if a.topo:
        default_topo = ftar.topo(a.topo, a.lonely, nranks=world)
    elif os.environ.get("FT_TOPO") or os.environ.get("FT_LONELY", "0") not in ("", "0"):
        default_topo = ftar.topo_from_env(world, bucket)
    else:
        default_topo = ftar.exec_choose(world, bucket, chunk_bytes=a.chunk_bytes or None).topo
    default_chunk = a.chunk_bytes   # 0: the model's piece, per call

    def model_chunk(t, form):
        """the model's piece for (topology, form) under the constants set now, as explicit bytes (a whole
        block when the model takes whole blocks)"""
        try:
            c = ftar.exec_choose(world, bucket, topo_=t, form=form).chunk_bytes
        except ftar.FtarError:   # a form whose rate is unmeasured (the collective): its reduce-scatter's piece
            c = ftar.exec_choose(world, bucket, topo_=t, form="direct").chunk_bytes
        return c or -(-n // world) * esz
    err = ""
    hung = False
    if not a.host_comm:
        phase("rccl preflight")
        err = preflight(float(os.environ.get("FTAR_BENCH_PREFLIGHT_S", "60")))
        hung = "not complete" in err
        flag = torch.tensor([1 if hung else 0], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        if flag.item():   # some rank's RCCL work may never finish: never wait on the whole device again,
            sync_state["device"] = False
            # and leave its stream: everything from here on (ftar calls, torch ops, sync()) runs on a fresh
            # one, so nothing queues behind the call that never completed
            stream = torch.cuda.Stream(device=dev)
            torch.cuda.set_stream(stream)
        phase("default")
    try:
        if err:
            raise RuntimeError(err)
        if os.environ.get("FTAR_BENCH_FAIL_DEFAULT") and not a.host_comm:   # rehearses the fallback below
            raise RuntimeError("FTAR_BENCH_FAIL_DEFAULT set")
        fn_default = run_with(default_topo, default_chunk, base_form)
        ms_default = timed(fn_default, a.steps, a.warmup)
        ok_default, why_default = check_y(fn_default)
    except Exception as e:  # noqa: BLE001
        if a.host_comm:
            raise
        err = str(e)[:200]
    bad = torch.tensor([1 if err else 0], dtype=torch.int32)
    dist.all_reduce(bad, op=dist.ReduceOp.MAX)   # every rank takes the same path
    if bad.item():
        # the first RCCL p2p transfers of the run failed: the IPC peer forms over a host-bootstrapped
        # communicator still move the data over xGMI, so the run keeps a measured line (the broken RCCL
        # communicator is left alone: destroying it could block)
        rccl_ranks = all_errors(err)
        state["rccl_ranks"] = rccl_ranks
        rccl_error = f"default configuration over RCCL failed: {err or 'on another rank'}"
        sys.stderr.write(f"[bench rank {rank}] {rccl_error}; falling back to the host-bootstrapped peer forms\n")
        a.host_comm = True
        comm = ftar.dist.init_host_comm(device=local)
        base_form = "peer-read"
        default_chunk = a.chunk_bytes
        fn_default = run_with(default_topo, default_chunk, base_form)
        ms_default = timed(fn_default, a.steps, a.warmup)
        ok_default, why_default = check_y(fn_default)
    if state.get("preflight_ev") is not None and not sync_state["device"]:
        # the rehearsal's proof that the fallback ran beside the stuck stream, not behind it
        state["stuck_stream_still_blocked"] = not state["preflight_ev"].query()
    ran = comm.last_exec()   # what the model chose for the default configuration (form "auto")
    default_info = {"topology": str(default_topo), "chunk_bytes": default_chunk, "form": base_form,
                    "ran": ran, "ms": round(ms_default, 4), "busbw_GBps": round(bws(ms_default)[1], 2),
                    "enqueue_ms": enq["ms"], "check": "ok" if ok_default else f"MISMATCH ({why_default})"}
    state["line"] = make_result(ms_default, default_topo, default_chunk, base_form, ok_default, a.steps, a.warmup,
                                {"config_selection": "default (sweep not reached)", "default_config": default_info})
    if "stuck_stream_still_blocked" in state:
        state["line"]["fallback_stream"] = {"fresh": True,
                                            "stuck_stream_still_blocked": state["stuck_stream_still_blocked"]}

    # 2. the sweep: every factorization of P and the ring x chunk sizes x form, in tiers (below)
    phase("sweep core")
    sweep = []
    cands = [str(default_topo)] + (["1"] if world > 1 else []) + [",".join(map(str, f)) for f in _factorizations(world)]
    seen, plan = set(), []
    for tp in cands:
        t = ftar.topo("1" if tp == "ring" else tp, 0 if "+" not in tp else int(tp.split("+")[1]))
        key = str(t)
        if key in seen:
            continue
        seen.add(key)
        forms = ["direct"] + (["collective"] if (not t.ring and n % world == 0) else []) + ["stages"]
        if a.host_comm:  # the host-bootstrapped communicator has no p2p transfers: the peer forms only
            forms = []
        for form in forms:
            mc = model_chunk(t, form)   # the model's piece for this topology and form (default constants)
            chunks = {4 << 20, 16 << 20, 64 << 20, mc}
            if key == str(default_topo) and form == "direct":  # 256 KiB ... 64 MiB
                chunks |= {256 << 10, 1 << 20}
                plan.append((t, mc, "direct:ncclreg"))
            if form == "stages" and t.ring:
                chunks = {mc}  # the reference's ring rounds: one point is enough
            plan += [(t, chunk, form) for chunk in sorted(chunks)]
        if not a.no_peer and t.lonely == 0:  # no pieces: whole-block kernels
            plan += [(t, 0, f) for f in ("peer-read", "peer-write", "peer-read-reg", "peer-write-reg")]
            if key == str(default_topo):  # copy policy and fold kernel over xGMI (same bits)
                plan += [(t, 0, f) for f in ("peer-read-reg:plain", "peer-write-reg:plain",
                                                         "peer-read-reg:vec", "peer-write-reg:vec",
                                                         "peer-read-reg:dma", "peer-write-reg:dma", "peer-read:dma")]
    # stable sort into tiers, so the likeliest winners are timed before the budget can run out: the default
    # topology's direct RCCL forms and the ring's (c4_ring, BASELINE configs[3]), then the default topology's
    # peer forms, the other topologies' direct/collective forms, the reference's staged rounds, the other peer
    # forms.  Tier 0 is the required "sweep core" stage; the rest runs after C5 and the host-memory rate, in
    # whatever time the budget leaves (DIST_STAGES, StageClock)
    def tier(p):
        t, _, form = p
        default = str(t) == str(default_topo)
        if form.startswith("peer-"):
            return 1 if default else 4
        if form.startswith("direct"):
            return 0 if default or t.ring else 2
        return 2 if form == "collective" else 3
    plan.sort(key=tier)
    clock = StageClock(budget, t_start)
    state["clock"] = clock

    def agreed(name):
        """rank 0's decision whether the stage runs, and its time limit, on every rank (the ranks' clocks
        differ by their start-up times; a stage some rank skipped would leave the others in its collectives)"""
        v = torch.tensor([1.0 if clock.may_run(name) else 0.0, clock.limit(name)], dtype=torch.float64)
        dist.broadcast(v, 0)
        return bool(v[0].item()), v[1].item()

    def xgmi_probe_stage(limit_s):
        """xGMI calibration: link rates by copy kernels (read/write, one peer / all peers), every rank at once,
        min/max over ranks; the workgroup-cap sweep only if the first pass left time for it (the loopback
        rehearsal's probe took 40 s on one shared GPU); then the model's fit from it"""
        t0 = time.time()
        try:
            pr = comm.xgmi_probe(64 << 20, iters=10)
            vals = torch.tensor(list(pr.values()), dtype=torch.float64)
            lo, hi = vals.clone(), vals.clone()
            dist.all_reduce(lo, op=dist.ReduceOp.MIN)
            dist.all_reduce(hi, op=dist.ReduceOp.MAX)
            state["line"]["xgmi_probe_GBps"] = {k: [round(lo[i].item(), 1), round(hi[i].item(), 1)]
                                                for i, k in enumerate(pr)}
            state["line"]["xgmi_probe_GBps"]["note"] = ("[min, max] over ranks; 64 MiB per peer per copy, "
                                                        "10 launches, all ranks at once")
            first = torch.tensor([time.time() - t0], dtype=torch.float64)
            dist.broadcast(first, 0)   # every rank takes the same decision
            if 2.5 * first.item() < limit_s:
                # how many CUs fill the links: the same copies capped at w workgroups (256 threads) per peer
                by_cap = {}
                for w in (4, 8, 16, 32, 64):
                    pc = comm.xgmi_probe(64 << 20, iters=5, wg_per_peer=w)
                    v = torch.tensor([pc["read_all_peers"], pc["write_all_peers"]], dtype=torch.float64)
                    dist.all_reduce(v, op=dist.ReduceOp.MIN)
                    by_cap[w] = {"read_all_peers": round(v[0].item(), 1), "write_all_peers": round(v[1].item(), 1)}
                state["line"]["xgmi_probe_GBps"]["by_workgroups_per_peer"] = by_cap
                # where a capped copy beat the uncapped one by > 10 % on every rank, the peer forms get a
                # sweep entry with that cap (the same decision on every rank: the rates are MIN-reduced)
                extra = probe_cap_entries(state["line"]["xgmi_probe_GBps"], by_cap)
                rest[0:0] = [(default_topo, 0, f) for f in extra if not a.no_peer]
            else:
                state["line"]["xgmi_probe_GBps"]["by_workgroups_per_peer"] = {
                    "skipped": f"first pass took {first.item():.1f}s of a {limit_s:.0f}s stage limit"}
        except Exception as e:  # noqa: BLE001
            state["line"]["xgmi_probe_GBps"] = {"error": str(e)[:200]}
        try:
            state["line"]["cost_model_fit"] = fit_cost_model(state["line"].get("xgmi_probe_GBps"))
        except Exception as e:  # noqa: BLE001
            state["line"]["cost_model_fit"] = {"error": str(e)[:200]}

    def sweep_run(entries, limit_s, what):
        """time `entries` in order until `limit_s` seconds have gone (rank 0's clock, broadcast)"""
        t0 = time.time()
        for i, (t, chunk, form) in enumerate(entries):
            stop = torch.tensor([1 if time.time() - t0 > limit_s else 0], dtype=torch.int32)
            dist.broadcast(stop, 0)  # every rank takes the same decision
            if stop.item():
                sweep.append({"skipped": f"{what}: its {limit_s:.0f}s reached ({len(entries) - i} entries left)"})
                return
            key = str(t)
            phase(f"sweep {key} {form} {chunk}", major=False)
            try:
                fn = run_with(t, chunk, form)
                ms_ = timed(fn, steps=min(5, a.steps), warmup=1)
                ok_, why_ = check_y(fn)   # every configuration's own output, before it may be chosen
            except Exception as e:  # noqa: BLE001  one bad configuration must not end the run
                sweep.append({"topology": key, "chunk_bytes": chunk, "form": form, "error": str(e)[:200]})
                continue
            sweep.append({"topology": key, "chunk_bytes": chunk, "form": form, "ms": round(ms_, 4),
                          "busbw_GBps": round(bws(ms_)[1], 2), "enqueue_ms": enq["ms"],
                          "check": "ok" if ok_ else f"MISMATCH ({why_})"})

    core = [p for p in plan if tier(p) == 0]
    rest = [p for p in plan if tier(p) > 0]
    state["line"]["sweep"] = sweep
    sweep_run(core, min(sweep_budget, agreed("sweep core")[1]), "sweep core")
    phase("xgmi probe")
    go, lim = agreed("xgmi probe")
    if world > 1 and go:
        xgmi_probe_stage(lim)

    # BASELINE configs[4] (C5): bf16 bucket of 2^29 elements (1 GiB) with the cost model's topology (fitted to
    # the probe when it ran), the default data movement, and every other width; validated like the rest
    phase("C5 bf16")
    if a.dtype == "f32" and not a.no_c5:
        try:
            state["line"]["c5_bf16"] = measure_c5()
        except Exception as e:  # noqa: BLE001
            state["line"]["c5_bf16"] = {"error": str(e)[:200]}

    # the host-memory end-to-end rate: PCIe in and out included, never the headline
    phase("host e2e")
    if not a.no_host:
        try:
            state["line"]["host_e2e"] = measure_host()
        except Exception as e:  # noqa: BLE001
            state["line"]["host_e2e"] = {"error": str(e)[:200]}

    # the rest of the sweep, in the time the later required stages leave
    phase("sweep rest")
    go, lim = agreed("sweep rest")
    if go:
        sweep_run(rest, min(sweep_budget, lim), "sweep rest")
    else:
        sweep.append({"skipped": f"sweep rest: {len(rest)} entries, no time left in the budget"})
    state["line"]["sweep"] = sweep

    # the execution model against this run's own sweep: every entry's prediction under
    # the constants the probe gave, the p2p constants re-fitted to the measured times (issue measured
    # directly from the enqueue times), and the re-fitted model's choice timed next to the sweep's best
    phase("cost model")
    try:
        state["line"]["cost_model"] = validate_model(sweep)
        if a.save_cost and rank == 0:   # the node's calibration, for FTAR_COST_FILE
            ftar.cost_save(a.save_cost)
            state["line"]["cost_model"]["saved_to"] = a.save_cost
    except Exception as e:  # noqa: BLE001  the model's report must not cost the run its line
        state["line"]["cost_model"] = {"error": str(e)[:200]}

    # 3. the sweep's best validated configuration, re-timed like the default, if it is faster
    phase("headline")
    ok_runs = [r for r in sweep if "ms" in r and r.get("check") == "ok"]
    best = min(ok_runs, key=lambda r: r["ms"]) if ok_runs else None
    if best is not None and best["ms"] < ms_default:
        best_topo = ftar.topo("1" if best["topology"] == "ring" else best["topology"])
        fn_best = run_with(best_topo, best["chunk_bytes"], best["form"])
        ms = timed(fn_best, a.steps, a.warmup)
        ok, _ = check_y(fn_best)
        if ok and ms < ms_default:
            carry = {k: state["line"][k] for k in ("xgmi_probe_GBps", "cost_model_fit", "cost_model", "fallback_stream",
                                                   "c5_bf16", "host_e2e") if k in state["line"]}
            state["line"] = make_result(ms, best_topo, best["chunk_bytes"], best["form"], ok, a.steps, a.warmup,
                                        {"config_selection": "best validated configuration of the sweep",
                                         "default_config": default_info, "sweep": sweep, **carry})
        else:
            state["line"]["config_selection"] = "default (sweep best not faster when re-timed)"
    else:
        state["line"]["config_selection"] = "default (fastest validated configuration)"
    # the roofline again, now with the probe's per-link rate (frac_of_probe) if the sweep reached the probe
    hl = state["line"]
    hl["roofline"] = allreduce_roofline(world, torch.cuda.device_count(), bucket, hl["ms_per_step"],
                                        hl["config"]["xgmi_links"],
                                        link_rate_from_probe(hl.get("xgmi_probe_GBps"), world))
    # north_star's transport is RCCL point-to-point: its best validated configuration is graded on its own,
    # whatever form won the headline
    if not a.host_comm:
        hl["rccl_p2p_best"] = rccl_p2p_best(sweep + [{**default_info, "check": "ok" if ok_default else "x",
                                                      "form": default_info["ran"]["form"],
                                                      "chunk_bytes": default_info["ran"]["chunk_bytes"]}],
                                            world, torch.cuda.device_count(), bucket,
                                            lambda r: links_driven(world, r["topology"], r["form"]))
        if hl["rccl_p2p_best"] is not None:
            hl["rccl_p2p_best"]["is_headline"] = all(hl["config"][f] == hl["rccl_p2p_best"][f]
                                                     for f in ("form", "topology", "chunk_bytes"))
        # BASELINE configs[3] says "ring AllReduce ... chunk size swept": the ring topology's best entry in
        # each RCCL form, labelled, so nobody reads the gather as a ring (DESIGN §9 names the one the >= 70 %
        # xGMI target is judged on: the direct form, the reference ring's bits over all links)
        hl["c4_ring"] = c4_ring_by_form(sweep, world, torch.cuda.device_count(), bucket,
                                        lambda r: links_driven(world, r["topology"], r["form"]))

    # phase timelines (rank 0's view) of the default and of the fastest validated configuration of each form:
    # where a call's time goes (transfer rounds vs folds vs barriers), for the next round's tuning
    phase("phase timing")
    try:
        go, lim = agreed("phase timing")
        if not go:
            raise RuntimeError(f"skipped: {lim:.0f}s left after the required stages")
        fam_best = {}
        for r in ok_runs:
            if r["form"] not in fam_best or r["ms"] < fam_best[r["form"]]["ms"]:
                fam_best[r["form"]] = r
        configs = [("default", default_topo, default_chunk, base_form)] + [
            (f"best {fam}", ftar.topo("1" if r["topology"] == "ring" else r["topology"]), r["chunk_bytes"], fam)
            for fam, r in sorted(fam_best.items())]
        phases = {}
        comm.phase_timing(True)
        for label, t, ch, form in configs:
            fn = run_with(t, ch, form)
            fn()
            sync()
            phases[label] = {"topology": str(t), "chunk_bytes": ch, "form": form, "phases_ms": comm.last_phases()}
        comm.phase_timing(False)
        state["line"]["phases_rank0"] = phases
    except Exception as e:  # noqa: BLE001
        state["line"]["phases_rank0"] = {"error": str(e)[:200]}

    # 4. RCCL's own ncclAllReduce on the same communicator and bucket (yardstick)
    phase("rccl yardstick")
    try:
        go, lim = agreed("rccl yardstick")
        if not go:
            raise RuntimeError(f"skipped: {lim:.0f}s left after the required stages")
        y2 = torch.empty_like(x)
        ms_rccl = timed(lambda: comm.rccl_allreduce(x, y2, n, a.dtype, "sum", stream=stream), min(a.steps, 10), 2)
        del y2
        state["line"]["rccl_native_allreduce"] = {"ms": round(ms_rccl, 4), "busbw_GBps": round(bws(ms_rccl)[1], 2)}
    except Exception as e:  # noqa: BLE001
        state["line"]["rccl_native_allreduce"] = None
        sys.stderr.write(f"rccl yardstick failed: {e}\n")

    # BASELINE configs[2] quotes 2 GPUs on a 256 MiB bucket: the headline configuration on the first 2^26
    # elements of the same buffers, as a line item (the headline keeps the 1 GiB bucket at every N: weak scaling)
    phase("256 MiB")
    try:
        n2 = min(n, 1 << 26)
        go, lim = agreed("256 MiB")
        if n2 < n and not go:
            state["line"]["bucket_256MiB"] = {"skipped": f"{lim:.0f}s left"}
        elif n2 < n:
            hb = state["line"]["config"]
            t2 = ftar.topo("1" if hb["topology"] == "ring" else hb["topology"])
            f2 = run_with(t2, hb["chunk_bytes"], hb["form"])
            xin2, yout2 = f2.xin[:n2], f2.yout[:n2]
            ms2 = timed(lambda: comm.allreduce(xin2, yout2, n2, a.dtype, "sum", topo_=t2, stream=stream),
                        min(a.steps, 10), 2)
            alg2 = n2 * esz / (ms2 * 1e-3) / 1e9
            state["line"]["bucket_256MiB"] = {
                "topology": str(t2), "form": hb["form"], "chunk_bytes": hb["chunk_bytes"], "ms": round(ms2, 4),
                "value_GBps": round(world * alg2, 2), "algbw_GBps_per_rank": round(alg2, 2),
                "busbw_GBps_per_rank": round(alg2 * 2 * (world - 1) / world if world > 1 else alg2, 2)}
    except Exception as e:  # noqa: BLE001
        state["line"]["bucket_256MiB"] = {"error": str(e)[:200]}

    # 7. the reference's own CPU/MPI path on this node's host cores, in the same run (north_star): its ring
    # over MPICH with P ranks (oracle/_ref/ref_golden arbench: mpi_mod.hpp's MPI_Allreduce_FT, 14 OpenMP
    # threads per rank), on a bounded sample, rank 0 only while the other ranks wait
    phase("reference cpu/mpi")
    go, _ = agreed("reference cpu/mpi")
    if rank == 0 and not a.no_cpu_baseline and go:
        state["line"]["reference_cpu_mpi"] = reference_mpi_path(world)
    dist.barrier()

    phase("end")
    state["line"]["stage_wall_s"] = dict(stage_t)
    state["line"]["stages_skipped_for_budget"] = dict(clock.skipped)
    state["line"]["budget_s"] = budget
    state["line"]["wall_s"] = round(time.time() - t_start, 1)
    emit(state["line"])
    state["done"] = True
    unblock()
    if not sync_state["device"]:
        # an RCCL kernel that never completed is still on the device: tearing the runtime down would wait
        # for it, so the line printed above is this process's last act
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)
    for i in reg.get("ids", []):
        comm.deregister(i)
    comm.destroy()
    dist.destroy_process_group()


def main():
    a = parse()
    if a.engine_local_only:   # one line item alone (under rocprofv3: the engine's kernel timeline)
        print(json.dumps({"engine_local": engine_local(steps=a.steps, warmup=a.warmup,
                                                       chunk_bytes=a.chunk_bytes or None)}), flush=True)
    elif int(os.environ.get("WORLD_SIZE", "1")) > 1 or a.force_dist:
        bench_distributed(a)
    else:
        bench_single(a)


if __name__ == "__main__":
    main()
