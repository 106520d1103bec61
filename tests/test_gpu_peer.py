"""Peer-direct data movement (ftar_comm_set_peer_direct), both forms: "read" (the plan's fold reads the
other ranks' exchange buffers directly, the all-gather pulls every final block) and "write" (every rank
pushes its copies into the owners' buffers, folds locally, pushes its final block); barriers are
stream-ordered.

* in-process groups on cuda:0 (local transport: the peers' buffers are plain pointers): every golden
  case, the one-round ring and trees, ragged and larger buckets, all bit-exact vs the oracle; plans
  that are not one-round (lonely ranks, staged forms) fall back to the RCCL-style executor;
* the IPC primitive itself across two processes on one device (dmabuf IPC, what RcclTransport
  uses to map peers on other GPUs): process B reduces through a mapping of process A's buffer.
"""
import ctypes

import numpy as np
import pytest
import torch.multiprocessing as mp

import ftar_inputs as fi
import golden_cases as gc
import oracle_lib
from gpu_util import filled_dev, from_dev, to_dev

pytestmark = pytest.mark.gpu

_groups = {}


def group(P):
    import ftar
    if P not in _groups:
        _groups[P] = ftar.Comm.init_local(P)
    return _groups[P]


def run_peer(ins, topo, lonely=0, dtype=6, op=0, outofplace=False, ag="direct", rs="direct", repeat=1, mode="read",
             registered=False):
    g = group(len(ins))
    g.set_peer_direct(mode)
    g.set_allgather(ag)
    g.set_reduce_scatter(rs)
    regs = []
    try:
        n = ins[0].size
        send = [to_dev(x) for x in ins]
        recv = [filled_dev(x.nbytes) for x in ins] if outofplace else send
        if registered:   # every rank's send and recv buffers: the in-place (no local pass) paths
            nb = max(1, ins[0].nbytes)
            regs.append(g.register([p for _, p in send], nb))
            if outofplace:
                regs.append(g.register([p for _, p in recv], nb))
        for it in range(repeat):
            sb = [p for _, p in send] if outofplace else None
            g.allreduce(sb, [p for _, p in recv], n, dtype, op, topo_=topo, lonely=lonely)
            if outofplace and it + 1 < repeat:
                send, recv = recv, send
        return [from_dev(t, ins[0].dtype, n) for t, _ in recv]
    finally:
        for ids in regs:
            g.deregister(ids)
        g.set_peer_direct(False)


MODES = ["read", "write"]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("case", gc.allreduce_cases(max_n=70000), ids=lambda c: c["id"])
def test_peer_direct_matches_reference_golden(case, mode):
    ins = gc.case_inputs(case)
    outs = run_peer(ins, case["topo"], case["lonely"], case["dtype"], case["op"], case["outofplace"],
                    repeat=case["repeat"], mode=mode)
    for r in range(case["P"]):
        gc.check_output(case, r, outs[r])


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("dt", ["f32", "bf16", "f64", "i16"])
@pytest.mark.parametrize("P,topo", [(2, "1"), (8, "1"), (5, "1"), (8, "8"), (8, "2,4"), (8, "2,2,2"), (9, "3,3"),
                                    (16, "4,4"), (16, "2,2,2,2")])
def test_peer_direct_one_round_plans(P, topo, dt, mode):
    n = 40_009 * P + 3       # ragged blocks, unaligned block offsets
    ins = [fi.fill(dt, 9, r, n) for r in range(P)]
    outs = run_peer(ins, topo, dtype=fi.BY_NAME[dt], mode=mode)
    ref = oracle_lib.allreduce(ins, topo, dtype=fi.BY_NAME[dt])
    for r in range(P):
        assert outs[r].tobytes() == ref[r].tobytes(), r


@pytest.mark.parametrize("P,topo,lonely,form", [(5, "2,2", 1, "direct"), (8, "2,4", 0, "stages"),
                                                (8, "1", 0, "stages")])
@pytest.mark.parametrize("mode", MODES)
def test_peer_direct_falls_back_for_multi_round_plans(P, topo, lonely, form, mode):
    n = 30_001
    ins = [fi.fill("f32", 10, r, n) for r in range(P)]
    outs = run_peer(ins, topo, lonely, ag=form, rs=form, mode=mode)
    ref = oracle_lib.allreduce(ins, topo, lonely)
    for r in range(P):
        assert outs[r].tobytes() == ref[r].tobytes(), r


def test_peer_direct_growing_buckets_and_mode_switches():
    """Exchange buffers regrow (unmap, free, remap) and calls alternate with the p2p executor."""
    import ftar
    P = 4
    g = group(P)
    for i, n in enumerate((1000, 200_003, 7, 600_001, 90_001)):
        ins = [fi.fill("f32", 11, r, n) for r in range(P)]
        ref = oracle_lib.allreduce(ins, "2,2")
        for mode in (MODES if i % 2 else MODES[::-1]):   # the two forms share (and regrow) the buffers
            outs = run_peer(ins, "2,2", mode=mode)
            assert all(outs[r].tobytes() == ref[r].tobytes() for r in range(P)), (n, mode)
        g.set_chunk_bytes(4096)
        bufs = [to_dev(x) for x in ins]
        g.allreduce(None, [p for _, p in bufs], n, "f32", topo_="2,2")
        assert all(from_dev(t, np.float32, n).tobytes() == ref[r].tobytes() for r, (t, _) in enumerate(bufs)), n
    assert not g[0].peer_direct and isinstance(ftar.Comm.peer_direct, property)


# ---- the IPC primitive across processes ---------------------------------------------------------
def _ipc_owner(n, q_handle, q_done):
    import sys, os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "allreduce-over-mpi_amd"), os.path.join(root, "tests")]
    import ftar  # noqa: F401  (loads the HIP runtime torch uses)
    import ftar_inputs as fi
    hip = ctypes.CDLL("libamdhip64.so.7")
    lib = ftar.lib()
    p = ctypes.c_void_p()
    assert hip.hipSetDevice(0) == 0
    inner = 4112   # export a pointer INSIDE the allocation (a registered tensor): handle + offset
    assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(n * 4 + inner)) == 0
    x = fi.fill("f32", 12, 0, n)
    px = ctypes.c_void_p(p.value + inner)
    assert hip.hipMemcpy(px, x.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(n * 4), 1) == 0   # H2D
    h = ctypes.create_string_buffer(128)
    lib.ftar_debug_ipc_handle.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    assert lib.ftar_debug_ipc_handle(px, h) == 0
    q_handle.put(h.raw)
    ok = q_done.get(timeout=240)
    assert hip.hipFree(p) == 0
    q_handle.put(("owner", ok))


def _ipc_user(n, q_handle, q_done, q_res):
    import sys, os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "allreduce-over-mpi_amd"), os.path.join(root, "tests")]
    import ftar
    import ftar_inputs as fi
    import torch
    try:
        raw = q_handle.get(timeout=240)
        lib = ftar.lib()
        lib.ftar_debug_ipc_open.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]
        lib.ftar_debug_ipc_close.argtypes = [ctypes.c_void_p]
        h = ctypes.create_string_buffer(raw, 128)
        mapped = ctypes.c_void_p()
        assert lib.ftar_debug_ipc_open(h, ctypes.byref(mapped)) == 0
        mine = fi.fill("f32", 12, 1, n)
        t = torch.from_numpy(mine).cuda()
        out = torch.empty_like(t)
        ftar.reduce([mapped.value, t.data_ptr()], out.data_ptr(), n, "f32", "sum")
        torch.cuda.synchronize()
        exp = (fi.fill("f32", 12, 0, n) + mine).astype(np.float32)
        ok = out.cpu().numpy().tobytes() == exp.tobytes()
        assert lib.ftar_debug_ipc_close(mapped) == 0
        q_res.put(("user", ok))
    except Exception as e:  # report, don't hang the parent
        q_res.put(("user", repr(e)))
    finally:
        q_done.put(True)


def test_ipc_mapping_across_processes():
    ctx = mp.get_context("spawn")
    qh, qd, qr = ctx.Queue(), ctx.Queue(), ctx.Queue()
    n = (1 << 20) + 7
    a = ctx.Process(target=_ipc_owner, args=(n, qh, qd))
    b = ctx.Process(target=_ipc_user, args=(n, qh, qd, qr))
    a.start()
    b.start()
    res = qr.get(timeout=300)
    b.join(timeout=120)
    a.join(timeout=120)
    assert res == ("user", True), res
    assert a.exitcode == 0 and b.exitcode == 0


def test_rccl_peer_plumbing_single_rank():
    """RcclTransport's barrier (4-byte ncclAllReduce) and map_peers (IPC handle all-gather over RCCL) on a
    1-rank RCCL communicator: every call of the multi-GPU peer path except opening another rank's handle."""
    import ftar
    comm = ftar.Comm.init_rank(1, ftar.get_unique_id(), 0, 0)
    try:
        lib = ftar.lib()
        lib.ftar_debug_peer_selftest.argtypes = [ctypes.c_void_p]
        assert lib.ftar_debug_peer_selftest(comm.handle) == 0, lib.ftar_last_error()
        comm.peer_direct = True
        assert comm.peer_direct == 1
        comm.peer_direct = "write"
        assert comm.peer_direct == 2
        probe = comm.xgmi_probe(1 << 20, iters=2)   # 1 rank: only the local copy has a partner
        assert probe["local_copy"] > 0 and probe["read_all_peers"] == 0, probe
    finally:
        comm.destroy()


@pytest.mark.parametrize("P", [2, 8])
def test_xgmi_probe_local_group(P):
    """The calibration probe on an in-process group (every 'peer' is this GPU): every pattern runs, all
    ranks at once, and reports a rate."""
    import threading
    g = group(P)
    res = [None] * P

    def run(r):
        res[r] = g[r].xgmi_probe(1 << 20, iters=3)
    th = [threading.Thread(target=run, args=(r,)) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    for r in range(P):
        assert res[r] is not None and all(v > 0 for v in res[r].values()), (r, res[r])


def test_peer_write_in_place_and_out_of_place_repeats():
    """Write form: repeated calls reuse the slots and final areas with two barriers per call."""
    P, n = 8, 123_457
    ins = [fi.fill("f32", 13, r, n) for r in range(P)]
    for oop in (False, True):
        outs = run_peer(ins, "2,4", outofplace=oop, repeat=3, mode="write")
        exp = ins
        for _ in range(3):
            exp = oracle_lib.allreduce(exp, "2,4")
        for r in range(P):
            assert outs[r].tobytes() == exp[r].tobytes(), (oop, r)


@pytest.mark.parametrize("mode,topo,names", [
    (0, "2,2", ["start", "stage 0 moved", "stage 0 reduced", "stage 1 moved"]),
    ("read", "2,2", ["start", "copy-in", "barrier", "fold (remote reads)", "barrier", "gather (remote reads)",
                     "barrier"]),
    ("write", "4", ["start", "scatter (remote writes)", "barrier", "fold (local)", "push (remote writes)",
                    "barrier", "copy-out", "barrier"])])
def test_phase_timing(mode, topo, names):
    """ftar_comm_set_phase_timing / ftar_comm_phase_json: the phases of the last call, in issue order."""
    import threading
    P, n = 4, 1 << 20
    g = group(P)
    ins = [fi.fill("f32", 14, r, n) for r in range(P)]
    ref = oracle_lib.allreduce(ins, topo)
    for c in g.comms:
        c.phase_timing(True)
    try:
        outs = run_peer(ins, topo, mode=mode)
        got = [None] * P
        th = [threading.Thread(target=lambda r=r: got.__setitem__(r, g[r].last_phases())) for r in range(P)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=60)
    finally:
        for c in g.comms:
            c.phase_timing(False)
    assert all(outs[r].tobytes() == ref[r].tobytes() for r in range(P))
    for r in range(P):
        assert [p[0] for p in got[r]] == names, got[r]
        assert got[r][0][1] == 0.0 and all(ms >= 0 for _, ms in got[r]), got[r]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("case", [c for c in gc.allreduce_cases(max_n=70000) if c["n"] > 0][::3],
                         ids=lambda c: c["id"])
def test_peer_registered_matches_reference_golden(case, mode):
    """Registered buffers: the peer forms read the peers' inputs / write the peers' outputs in place."""
    ins = gc.case_inputs(case)
    outs = run_peer(ins, case["topo"], case["lonely"], case["dtype"], case["op"], case["outofplace"],
                    repeat=case["repeat"], mode=mode, registered=True)
    for r in range(case["P"]):
        gc.check_output(case, r, outs[r])


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("P,topo,dt", [(8, "1", "f32"), (8, "2,4", "bf16"), (8, "8", "f32"), (5, "1", "f64"),
                                       (16, "4,4", "f32")])
@pytest.mark.parametrize("oop", [False, True])
def test_peer_registered_one_round_plans(P, topo, dt, mode, oop):
    n = 50_021 * P + 5
    ins = [fi.fill(dt, 15, r, n) for r in range(P)]
    outs = run_peer(ins, topo, dtype=fi.BY_NAME[dt], mode=mode, registered=True, outofplace=oop, repeat=2)
    ref = oracle_lib.allreduce(oracle_lib.allreduce(ins, topo, dtype=fi.BY_NAME[dt]), topo, dtype=fi.BY_NAME[dt])
    for r in range(P):
        assert outs[r].tobytes() == ref[r].tobytes(), r


def test_peer_registered_phases_skip_the_local_pass():
    """With registered buffers the phase list has no copy-in / copy-out."""
    import ftar  # noqa: F401
    P, n = 4, 1 << 18
    g = group(P)
    ins = [fi.fill("f32", 16, r, n) for r in range(P)]
    for c in g.comms:
        c.phase_timing(True)
    try:
        names = {}
        for mode in MODES:
            run_peer(ins, "4", mode=mode, registered=True)
            names[mode] = [p[0] for p in g[0].last_phases()]
    finally:
        for c in g.comms:
            c.phase_timing(False)
    assert names["read"] == ["start", "barrier", "fold (remote reads)", "barrier", "gather (remote reads)",
                             "barrier"], names
    assert names["write"] == ["start", "scatter (remote writes)", "barrier", "fold (local)",
                              "push (remote writes)", "barrier"], names


@pytest.mark.parametrize("mode", ["read", "write"])
@pytest.mark.parametrize("nt,lds,dma", [(False, True, False), (True, False, False), (False, False, False),
                                        (True, True, True)])
@pytest.mark.parametrize("P,topo,dt", [(4, "4", "f32"), (8, "2,4", "f32"), (4, "1", "bf16"), (8, "8", "bf16")])
def test_peer_tuning_same_bits(mode, nt, lds, dma, P, topo, dt):
    """bench.py's peer tuning variants (plain copies, register-kernel fold, DMA-engine copies) change no bit: the fold's
    operands and order are the plan's either way ("2,4" folds nested)."""
    n = 200_003
    ins = [fi.fill(dt, 91, r, n) for r in range(P)]
    g = group(P)
    for c in g.comms:
        c.peer_tuning(nt=nt, lds=lds, dma=dma)
    try:
        got = run_peer(ins, topo, dtype=fi.BY_NAME[dt], mode=mode, registered=True, outofplace=True)
    finally:
        for c in g.comms:
            c.peer_tuning()
    ref = oracle_lib.allreduce(ins, topo, dtype=fi.BY_NAME[dt], outofplace=True)
    for r in range(P):
        assert np.array_equal(got[r].view(np.uint8), ref[r].view(np.uint8)), (r, mode, nt, lds)


@pytest.mark.parametrize("cap", [1, 4, 64])
@pytest.mark.parametrize("mode,registered", [("read", True), ("write", True), ("read", False), ("write", False)])
def test_peer_copy_cap_same_bits(cap, mode, registered):
    """bench.py's ":wgN" entries cap the peer forms' cross-GPU copies at N workgroups per segment (grid-stride
    beyond): same bytes, same bits."""
    P, topo, n = 4, "4", 300_007
    ins = [fi.fill("f32", 93, r, n) for r in range(P)]
    g = group(P)
    for c in g.comms:
        c.peer_wg_cap = cap
    try:
        got = run_peer(ins, topo, dtype=6, mode=mode, registered=registered, outofplace=True)
    finally:
        for c in g.comms:
            c.peer_wg_cap = 0
    ref = oracle_lib.allreduce(ins, topo, dtype=6, outofplace=True)
    for r in range(P):
        assert np.array_equal(got[r].view(np.uint8), ref[r].view(np.uint8)), (r, mode, cap)


@pytest.mark.parametrize("seed", range(3))
def test_random_soak_registered_subranges(seed):
    """Seeded random calls on SUB-RANGES of registered buffers (ftar_comm_register over a larger allocation,
    the call's buffers at the same offset on every rank, as ftar.h requires): the zero-copy peer paths map
    each peer's pointer as its registration base + my offset.  Random P, one-round topologies (ring, single
    stage, nested trees), dtypes, ops, ragged sizes, offsets, read/write, in place or out of place, and
    registrations of the input only, the output only, both, or a decoy registered first.  Bit-exact vs the
    oracle; a second call on the swapped buffers catches stale mappings."""
    import random

    import random_cases
    torch = __import__("torch")
    rng = random.Random(4000 + seed)
    for _ in range(int(__import__("os").environ.get("FTAR_SOAK", "100")) // 4):
        P = rng.choice([2, 3, 4, 6, 8])
        topo = rng.choice(["1"] + [",".join(map(str, f)) for f in random_cases.factorizations(P)])
        dt = rng.choice(["f32", "f32", "bf16", "f64", "i32", "u8", "i64"])
        op = "band" if dt in ("i32", "u8", "i64") and rng.random() < 0.3 else "sum"
        n = rng.choice([1, P - 1, P + 1, rng.randint(2, 5000), rng.randint(5000, 300_000)])
        off = rng.choice([0, 1, 3, 64, 1000])
        tail = rng.choice([0, 1, 4096])
        mode = rng.choice(["read", "write"])
        oop = rng.random() < 0.5
        which = rng.choice(["both", "both", "in", "out", "decoy"])
        dti, npdt = fi.BY_NAME[dt], fi.np_dtype(dt)
        esz = np.dtype(npdt).itemsize
        sd = rng.randint(0, 1 << 30)
        ins = [fi.fill(dt, sd, r, n) for r in range(P)]
        ref = oracle_lib.allreduce(ins, topo, 0, dti, 0 if op == "sum" else 1, outofplace=oop)
        ref2 = oracle_lib.allreduce(ref, topo, 0, dti, 0 if op == "sum" else 1, outofplace=oop)
        g = group(P)
        g.set_peer_direct(mode)
        g.set_allgather("direct")
        g.set_reduce_scatter("direct")
        total = (off + n + tail) * esz
        a = [to_dev(x, pad_elems=tail, offset_elems=off)[0] for x in ins]
        b = [torch.full((total,), 0xA5, dtype=torch.uint8, device="cuda") for _ in range(P)] if oop else a
        ids = []
        try:
            if which == "decoy":
                decoy = [torch.empty(4096, dtype=torch.uint8, device="cuda") for _ in range(P)]
                ids.append(g.register([t.data_ptr() for t in decoy], 4096))
            if which in ("both", "in", "decoy"):
                ids.append(g.register([t.data_ptr() for t in a], total))
            if oop and which in ("both", "out", "decoy"):
                ids.append(g.register([t.data_ptr() for t in b], total))
            if not oop and which == "out":
                ids.append(g.register([t.data_ptr() for t in a], total))
            pa = [t.data_ptr() + off * esz for t in a]
            pb = [t.data_ptr() + off * esz for t in b]
            g.allreduce(pa if oop else None, pb, n, dti, 0 if op == "sum" else 1, topo_=topo)
            got = [from_dev(t, npdt, n, off) for t in b]
            for r in range(P):
                assert got[r].tobytes() == ref[r].tobytes(), (P, topo, dt, op, n, off, mode, oop, which, r)
            # second call: the result as input (out of place: the buffers swap roles)
            g.allreduce(pb if oop else None, pa if oop else pb, n, dti, 0 if op == "sum" else 1, topo_=topo)
            got = [from_dev(t, npdt, n, off) for t in (a if oop else b)]
            for r in range(P):
                assert got[r].tobytes() == ref2[r].tobytes(), ("repeat", P, topo, dt, op, n, off, mode, oop, which, r)
        finally:
            for i in ids:
                g.deregister(i)
            g.set_peer_direct(False)
