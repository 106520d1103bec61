"""Peer-direct forms across real PROCESSES (one GPU, several processes): ftar_comm_init_host bootstraps
over a gloo group, the exchange buffers and registered buffers are mapped with IPC across the process
boundary (IpcRef: allocation handle + offset, refcounted imports) -- the machinery RcclTransport uses
between the GPUs of a node.  Every output is checked bit for bit against the oracle."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CASES = {2: [("1", 0, "stages", "stages", 1 << 16), ("2", 0, "direct", "collective", 0),
                 ("1", 0, "direct", "direct", 4096)],
             4: [("2,2", 0, "stages", "stages", 1 << 16), ("1", 0, "stages", "stages", 0),
                 ("2,2", 0, "direct", "collective", 1 << 15), ("4", 0, "direct", "direct", 0)],
             5: [("2,2", 1, "stages", "stages", 1 << 16), ("2,2", 1, "direct", "direct", 0)]}
CASES = {2: [("1", "f32"), ("2", "bf16"), ("1", "i16")],
         4: [("1", "f32"), ("2,2", "f32"), ("4", "bf16"), ("1", "i16")],
         5: [("1", "f32"), ("5", "bf16")]}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "allreduce-over-mpi_amd"), os.path.join(root, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    import ftar
    import ftar.dist
    import ftar_inputs as fi
    out = {}
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        comm = ftar.dist.init_host_comm(device=0)
        for topo, dt in CASES[world]:
            x = fi.fill(dt, 21, rank, n)
            xt = torch.from_numpy(x.view(np.uint8).copy()).cuda()
            for mode in ("read", "write"):
                for registered in (False, True):
                    for oop in (False, True):
                        src = xt.clone()
                        dst = torch.full_like(src, 0x5A) if oop else src
                        regs = []
                        if registered:
                            regs = [comm.register(src, src.numel())] + ([comm.register(dst, dst.numel())] if oop else [])
                        comm.peer_direct = mode
                        comm.allreduce(src if oop else None, dst, n, dt, "sum", topo_=topo)
                        torch.cuda.synchronize()
                        out[(topo, dt, mode, registered, oop)] = dst.cpu().numpy().tobytes()
                        for r in regs:
                            comm.deregister(r)
                        dist.barrier()
        # plans that need point-to-point transfers (staged forms, lonely ranks) are refused alike on every
        # rank before anything moves: the host-bootstrapped communicator has the peer forms only
        comm.peer_direct = 0
        xt = torch.from_numpy(fi.fill("f32", 23, rank, n).copy()).cuda()
        comm.reduce_scatter, comm.allgather = "stages", "stages"
        try:
            comm.allreduce(None, xt, n, "f32", "sum", topo_="1")
            out["p2p"] = "ran"
        except ftar.FtarError as e:
            out["p2p"] = e.status
        comm.reduce_scatter, comm.allgather = "direct", "direct"
        dist.barrier()
        comm.destroy()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001  report, don't hang the parent
        out["error"] = repr(e)
    q.put((rank, out))


@pytest.mark.parametrize("world", [2, 4, 5])
def test_peer_forms_across_processes(world):
    import ftar_inputs as fi
    import oracle_lib
    n = 100_003
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    for r in range(world):
        assert "error" not in res[r], res[r].get("error")
    for topo, dt in CASES[world]:
        ins = [fi.fill(dt, 21, r, n) for r in range(world)]
        ref = oracle_lib.allreduce(ins, topo, dtype=fi.BY_NAME[dt])
        keys = [k for k in res[0] if isinstance(k, tuple) and k[:2] == (topo, dt)]
        assert len(keys) == 8, keys
        for key in keys:
            for r in range(world):
                assert res[r][key] == ref[r].tobytes(), (world, key, r)
    assert all(res[r]["p2p"] == 2 for r in range(world)), [res[r]["p2p"] for r in range(world)]  # UNSUPPORTED


def _big_worker(rank, world, port, n, q):
    """Exchange-buffer growth across the 2 GiB line (tools/peer_rehearsal.py): the write form at n = 2^28 fp32
    needs a 2 GiB exchange buffer, and torch's HIP 7.0 runtime blocks forever in hipIpcOpenMemHandle for
    allocations whose size has bit 31 set; the buffer is sized around that (ipc_safe_size)."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "allreduce-over-mpi_amd"), os.path.join(root, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    import ftar
    import ftar.dist
    out = {}
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        comm = ftar.dist.init_host_comm(device=0)
        x = torch.full((n,), float(rank + 1), device="cuda")
        y = torch.empty_like(x)
        for mode in ("read", "write"):
            comm.peer_direct = mode
            comm.allreduce(x, y, n, "f32", "sum", topo_="1")
            torch.cuda.synchronize()
            out[mode] = bool((y == float(world * (world + 1) // 2)).all())
            y.zero_()
        # a 2 GiB registration is refused on every rank alike (no hang) where the runtime is affected
        big = torch.empty(1 << 29, dtype=torch.float32, device="cuda")
        try:
            r = comm.register(big, big.numel() * 4)
            comm.deregister(r)
            out["reg2g"] = "registered"
        except ftar.FtarError as e:
            out["reg2g"] = e.status
        comm.destroy()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        out["error"] = repr(e)
    q.put((rank, out))


def test_exchange_buffer_past_2gib():
    import torch
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    ps = [ctx.Process(target=_big_worker, args=(r, world, port, 1 << 28, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=100) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    for r in range(world):
        assert "error" not in res[r], res[r].get("error")
        assert res[r]["read"] and res[r]["write"], res[r]
    # agreed across ranks: both registered, or both refused with FTAR_ERR_HIP (the guard's agreed failure)
    assert res[0]["reg2g"] == res[1]["reg2g"], res
    affected = int(torch.version.hip.split(".")[0]) * 100 + int(torch.version.hip.split(".")[1]) < 702
    if affected and os.environ.get("FTAR_IPC_SIZE_GUARD", "") != "0":
        assert res[0]["reg2g"] != "registered", res


HOST_CASES = {2: [("1", "f32"), ("2", "bf16"), ("1", "i32")],
              3: [("3", "f32"), ("1", "f64")],
              4: [("2,2", "f32"), ("1", "bf16"), ("4", "u8")]}


def _host_worker(rank, world, port, n, q):
    """Host buffers on the host-bootstrapped communicator (the MPI drop-in's `ipc` transport): the read form
    piece by piece (peer_allreduce_host), 4 KiB and default pieces, pinned and pageable, in place and out of
    place, repeated; the write form keeps the whole-bucket path."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "allreduce-over-mpi_amd"), os.path.join(root, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    import ftar
    import ftar.dist
    import ftar_inputs as fi
    out = {}
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        comm = ftar.dist.init_host_comm(device=0)
        for topo, dt in HOST_CASES[world]:
            x = fi.fill(dt, 31, rank, n).view(np.uint8)
            for mode in ("read", "write"):
                comm.peer_direct = mode
                for piece in (4096, 0):
                    comm.host_chunk_bytes = piece
                    for pinned in (True, False):
                        for oop in (False, True):
                            def buf(init):
                                if pinned:
                                    b = torch.empty(init.size, dtype=torch.uint8, pin_memory=True).numpy()
                                    b[:] = init
                                    return b
                                return init.copy()
                            src = buf(x)
                            dst = buf(np.full_like(x, 0x5A)) if oop else src
                            for rep in range(2):  # a second call reuses the exchange buffer
                                if rep and not oop:
                                    src[:] = x
                                comm.allreduce_host(src if oop else None, dst, n, dt, "sum", topo_=topo)
                                torch.cuda.synchronize()
                            out[(topo, dt, mode, piece, pinned, oop)] = dst.tobytes()
                            dist.barrier()
            # 256-B pieces on a bucket that would need more than 1024 of them: the read form's
            # piece count is capped (every piece costs a host barrier), same bits
            if world == 2:
                comm.peer_direct = "read"
                comm.host_chunk_bytes = 256
                big = fi.fill(dt, 33, rank, 600_001).view(np.uint8)
                y = np.full_like(big, 0x5A)
                comm.allreduce_host(big, y, 600_001, dt, "sum", topo_=topo)
                torch.cuda.synchronize()
                out[("cap", topo, dt)] = y.tobytes()
                dist.barrier()
        comm.destroy()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001  report, don't hang the parent
        import traceback
        out["error"] = traceback.format_exc()
    q.put((rank, out))


@pytest.mark.parametrize("world", [2, 3, 4])
def test_host_buffers_across_processes(world):
    import ftar_inputs as fi
    import oracle_lib
    n = 70_001
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_host_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    for r in range(world):
        assert "error" not in res[r], res[r].get("error")
    for topo, dt in HOST_CASES[world]:
        ins = [fi.fill(dt, 31, r, n) for r in range(world)]
        ref = oracle_lib.allreduce(ins, topo, dtype=fi.BY_NAME[dt])
        keys = [k for k in res[0] if isinstance(k, tuple) and k[:2] == (topo, dt)]
        assert len(keys) == 16, keys
        for key in keys:
            for r in range(world):
                assert res[r][key] == ref[r].tobytes(), (world, key, r)
        if world == 2:
            big_ref = oracle_lib.allreduce([fi.fill(dt, 33, r, 600_001) for r in range(world)], topo,
                                           dtype=fi.BY_NAME[dt])
            for r in range(world):
                assert res[r][("cap", topo, dt)] == big_ref[r].tobytes(), (topo, dt, r)


SOAK_TOPOS = {2: ["1", "2"], 3: ["1", "3"], 4: ["1", "4", "2,2"]}
SOAK_DTYPES = ["f32", "bf16", "f64", "i32", "u8", "i16"]


def _soak_cases(world, count, seed):
    rng = np.random.default_rng(seed)
    cases = []
    for i in range(count):
        n = int(rng.choice([0, 1, 3, world - 1, world + 1, int(rng.integers(2, 5000)), int(rng.integers(5000, 300_000))]))
        cases.append((i, n, str(rng.choice(SOAK_DTYPES)), str(rng.choice(SOAK_TOPOS[world])),
                      int(rng.choice([256, 4096, 65536, 0])), bool(rng.integers(0, 2)), bool(rng.integers(0, 2))))
    return cases


def _soak_worker(rank, world, port, cases, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "allreduce-over-mpi_amd"), os.path.join(root, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    import ftar
    import ftar.dist
    import ftar_inputs as fi
    out = {}
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        comm = ftar.dist.init_host_comm(device=0)
        comm.peer_direct = "read"
        for i, n, dt, topo, piece, pinned, oop in cases:
            x = fi.fill(dt, 500 + i, rank, n).view(np.uint8)

            def buf(init):
                if pinned and init.size:
                    b = torch.empty(init.size, dtype=torch.uint8, pin_memory=True).numpy()
                    b[:] = init
                    return b
                return init.copy()
            src = buf(x)
            dst = buf(np.full_like(x, 0x5A)) if oop else src
            comm.host_chunk_bytes = piece
            comm.allreduce_host(src if oop else None, dst if dst.size else None, n, dt, "sum", topo_=topo)
            torch.cuda.synchronize()
            out[i] = dst.tobytes()
        dist.barrier()
        comm.destroy()
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        import traceback
        out["error"] = traceback.format_exc()
    q.put((rank, out))


@pytest.mark.parametrize("world", [2, 3, 4])
def test_host_buffers_random_soak(world):
    """The piece-pipelined host path on the host-bootstrapped communicator: 40 random cases per world size
    (empty and ragged buckets, six dtypes, ring and one-round trees, 256 B to auto pieces, pinned and
    pageable, in and out of place), bit-exact against the oracle"""
    import ftar_inputs as fi
    import oracle_lib
    cases = _soak_cases(world, 40, 1000 + world)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_soak_worker, args=(r, world, port, cases, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    for r in range(world):
        assert "error" not in res[r], res[r].get("error")
    for i, n, dt, topo, piece, pinned, oop in cases:
        ins = [fi.fill(dt, 500 + i, r, n) for r in range(world)]
        ref = oracle_lib.allreduce(ins, topo, dtype=fi.BY_NAME[dt])
        for r in range(world):
            assert res[r][i] == ref[r].tobytes(), (world, i, n, dt, topo, piece, pinned, oop, r)


def _mismatch_worker(rank, world, port, n, q):
    """Ranks whose host-path settings differ: the pipelined host path runs m + 2 host barriers and
    the whole-bucket path 3, so mismatched FTAR_HOST_PEER_PIPELINE / piece sizes / peer forms would pair
    barriers of different phases.  Every rank must get FTAR_ERR_INVALID_ARG from the same call, and the
    communicator must stay usable for the next, matched call."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "allreduce-over-mpi_amd"), os.path.join(root, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    import ftar
    import ftar.dist
    import ftar_inputs as fi
    out = {}
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        comm = ftar.dist.init_host_comm(device=0)
        x = fi.fill("f32", 41, rank, n)
        for what in ("piece", "form", "device_form"):
            comm.peer_direct = "read"
            comm.host_chunk_bytes = 0
            if what == "piece":
                comm.host_chunk_bytes = 4096 * (rank + 1)        # different piece sizes
            elif rank == 1:
                comm.peer_direct = "write"                       # read on rank 0, write on rank 1
            try:
                if what == "device_form":
                    xt = torch.from_numpy(x.copy()).cuda()
                    comm.allreduce(None, xt, n, "f32", "sum", topo_="1")
                    torch.cuda.synchronize()
                else:
                    y = x.copy()
                    comm.allreduce_host(None, y, n, "f32", "sum", topo_="1")
                    torch.cuda.synchronize()
                out[what] = "ran"
            except ftar.FtarError as e:
                out[what] = (e.status, "disagree" in str(e))
            dist.barrier()
        comm.peer_direct = "read"                                # matched again: the call works
        comm.host_chunk_bytes = 4096
        y = x.copy()
        comm.allreduce_host(None, y, n, "f32", "sum", topo_="1")
        torch.cuda.synchronize()
        out["after"] = y.tobytes()
        comm.destroy()
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        import traceback
        out["error"] = traceback.format_exc()
    q.put((rank, out))


def test_host_path_settings_must_agree_across_ranks():
    import ftar_inputs as fi
    import oracle_lib
    world, n = 2, 50_003
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_mismatch_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    for r in range(world):
        assert "error" not in res[r], res[r].get("error")
        for what in ("piece", "form", "device_form"):
            assert res[r][what] == (1, True), (r, what, res[r][what])
    ref = oracle_lib.allreduce([fi.fill("f32", 41, r, n) for r in range(world)], "1")
    for r in range(world):
        assert res[r]["after"] == ref[r].tobytes(), r


def _init_mismatch_worker(rank, world, port, q):
    """Ranks launched with different environments (FTAR_CHUNK_BYTES, FT_TOPO): communicator bring-up compares
    the settings that shape every rank's messages and fails on every rank, instead of a later call hanging."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "allreduce-over-mpi_amd"), os.path.join(root, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    import ftar
    import ftar.dist
    out = {}
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        for var, vals in (("FTAR_CHUNK_BYTES", ("1048576", "4194304")), ("FT_TOPO", ("1", "2"))):
            os.environ[var] = vals[rank % 2]
            try:
                comm = ftar.dist.init_host_comm(device=0)
                comm.destroy()
                out[var] = "initialised"
            except ftar.FtarError as e:
                out[var] = (e.status, "disagree" in str(e))
            del os.environ[var]
            dist.barrier()
        comm = ftar.dist.init_host_comm(device=0)   # alike again: fine
        comm.destroy()
        out["after"] = "ok"
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        import traceback
        out["error"] = traceback.format_exc()
    q.put((rank, out))


def test_mismatched_environments_fail_bring_up_on_every_rank():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_init_mismatch_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    for r in range(world):
        assert "error" not in res[r], res[r].get("error")
        assert res[r]["FTAR_CHUNK_BYTES"] == (1, True) and res[r]["FT_TOPO"] == (1, True), res[r]
        assert res[r]["after"] == "ok"
