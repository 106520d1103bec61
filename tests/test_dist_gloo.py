"""The N>1 path on the CPU: world_size 2..8 processes over gloo.

Each process builds ONLY its own rank's plan with libftar (exactly what
ftar_allreduce does on its GPU), then executes it with gloo point-to-point
messages instead of RCCL (same per-pair posting order), folding with the
pinned oracle's reduce (tests/plan_fold.py).  Every rank must end with the reference's golden
output: the independently compiled per-rank plans form a consistent
distributed protocol.  Also checks the unique-id bootstrap of ftar.dist.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, case_id, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "allreduce-over-mpi_amd"), os.path.join(root, "tests")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    import ftar
    import ftar.dist
    import golden_cases as gc
    import plan_fold

    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        uid = ftar.dist.exchange_unique_id()
        ids = [None] * world
        dist.all_gather_object(ids, uid)
        assert all(i == ids[0] for i in ids) and len(uid) == 128

        case = [c for c in gc.allreduce_cases() if c["id"] == case_id][0]
        x = gc.case_inputs(case)[rank]
        plan = ftar.plan_json(ftar.topo(case["topo"], case["lonely"]), world, rank, case["n"])
        bufs = {"src": x.copy(), "dst": x.copy(), "scratch": np.zeros(max(1, 2 * plan["scratch_half"]), x.dtype)}
        if case["outofplace"]:
            bufs["dst"] = np.frombuffer(b"\xa5" * x.nbytes, dtype=x.dtype).copy()
        for st in plan["stages"]:
            reqs = []
            for peer, buf, off, ln in st["sends"]:
                reqs.append(dist.isend(torch.from_numpy(bufs[buf][off:off + ln].copy()), dst=peer))
            incoming = []
            for peer, buf, off, ln in st["recvs"]:
                t = torch.empty(ln, dtype=torch.from_numpy(x[:1]).dtype)
                reqs.append(dist.irecv(t, src=peer))
                incoming.append((buf, off, ln, t))
            for r in reqs:
                r.wait()
            for buf, off, ln, t in incoming:
                bufs[buf][off:off + ln] = t.numpy()
            for it in st["reduces"]:
                off, ln = it["off"], it["len"]
                srcs = [np.ascontiguousarray(bufs[b][o:o + ln]) for b, o in it["srcs"]]
                bufs["dst"][off:off + ln] = plan_fold.fold(it, srcs, case["dtype"], case["op"])
        gc.check_output(case, rank, bufs["dst"])
        q.put((rank, "ok"))
    except Exception as e:  # report, don't hang the parent
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


CASES = ["ar_P2_t1_l0_f32_op0_n1003", "ar_P2_t2_l0_f32_op0_n65541", "ar_P4_t2-2_l0_f32_op0_n1003",
         "ar_P4_t1_l0_f32_op0_n17", "ar_P5_t2-2_l1_f32_op0_n1003", "ar_P4_t2-2_l0_f32_op0_n1003_oop",
         # the one-round forms at a node's size: direct ring and direct multi-stage trees, 8 processes
         "ar_P4_t2-2_l0_f64_op0_n1003", "ar_P8_t2-2-2_l0_f32_op0_n1003", "ar_P8_t2-4_l0_f32_op0_n65541",
         "ar_P8_t1_l0_f32_op0_n1003",
         # C5's width-8 tree and the other factorization of 8; a lonely rank at 7 and a 6-rank mixed radix
         "ar_P8_t8_l0_f32_op0_n65541", "ar_P8_t4-2_l0_f32_op0_n1003", "ar_P7_t2-3_l1_f32_op0_n1003",
         "ar_P6_t3-2_l0_f32_op0_n17"]


@pytest.mark.parametrize("case_id", CASES)
def test_distributed_plan_over_gloo(case_id):
    import golden_cases as gc
    case = [c for c in gc.allreduce_cases() if c["id"] == case_id][0]
    world = case["P"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case_id, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(v == "ok" for v in results.values()), results
