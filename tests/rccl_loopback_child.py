"""One rank of an RCCL communicator whose ranks share the box's one GPU (run under torchrun).

RCCL refuses two ranks of one communicator on the same device ("Duplicate GPU detected") only when their
host hashes are equal; NCCL_HOSTID gives every rank its own, so RCCL takes each rank for a separate node and
carries ncclSend/ncclRecv over its network transport (sockets on the loopback interface).  That is the
product's RcclTransport -- the replacement of handle_send/handle_recv (mpi_mod.hpp:1254-1305) -- executing
between ranks, on one GPU: the same plans, streams, pieces and kernels as over xGMI, only the wire differs.

Checks, per rank (written as one JSON line "LOOPBACK {...}"):
  * every golden case of this world size, all dtypes/ops/lonely layouts, in the three all-gather forms
    (direct, the reference's stages, collective): the reference's output bits (sha256 per rank);
  * a larger ragged bucket against the pinned oracle (ring and the widest tree), device and host buffers;
  * bf16 and RCCL's own ncclAllReduce on the same communicator.
FTAR_LOOPBACK_MODE=capture instead captures the AllReduce into a HIP graph and replays it (capture());
FTAR_LOOPBACK_MODE=soak runs seeded random cases with random per-call settings (soak());
FTAR_LOOPBACK_MODE=ddp trains through DistributedDataParallel with ftar's comm hook (ddp());
FTAR_LOOPBACK_MODE=full runs BASELINE's C4 and C5 buckets (full_size()).
FTAR_LOOPBACK_MODE=first_contact: rank 0 calls while the others never do (first_contact()).
"""
import json
import os
import sys
import traceback

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "allreduce-over-mpi_amd"))


def loopback_env(rank):
    """RCCL settings that let ranks on one GPU form a communicator (every rank its own 'host')."""
    os.environ["NCCL_HOSTID"] = f"ftar-loopback-{rank}"
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")


def main():
    import faulthandler
    faulthandler.enable()   # a crash inside the runtime still names the Python line it came from
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    loopback_env(rank)
    if os.environ.get("FTAR_LOOPBACK_LATE_RANK") == str(rank):   # write_race: this rank's copy-outs run late
        os.environ["FTAR_DEBUG_PEER_LATE_US"] = "150000"
    import numpy as np
    import torch
    import torch.distributed as dist

    import ftar
    import ftar.dist as fdist
    import ftar_inputs as fi
    import golden_cases as gc
    import oracle_lib
    from gpu_util import filled_dev, from_dev, to_dev

    max_n = int(os.environ.get("FTAR_LOOPBACK_MAX_N", "70000"))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    res = {"rank": rank, "world": world, "golden": 0, "oracle": 0, "fail": []}
    comm = fdist.init_comm(device=0)
    res["rccl"] = True

    def run(x, topo, lonely, dtype, op, outofplace, repeat=1, host=False, pinned=True):
        n = x.size
        if host:
            pin = (lambda t: t.pin_memory()) if pinned else (lambda t: t)
            send = pin(torch.from_numpy(x.copy())) if outofplace else None
            recv = pin(torch.from_numpy(x.copy())) if not outofplace else pin(torch.empty_like(torch.from_numpy(x)))
            for _ in range(repeat):
                comm.allreduce_host(send.data_ptr() if send is not None else None, recv.data_ptr(), n, dtype, op,
                                    topo_=topo, lonely=lonely)
            torch.cuda.synchronize()
            return recv.numpy().copy()
        s_t, s_p = to_dev(x)
        if outofplace:
            r_t, r_p = filled_dev(x.nbytes)
        else:
            r_t, r_p = s_t, s_p
        for it in range(repeat):
            comm.allreduce(s_p if outofplace else None, r_p, n, dtype, op, topo_=topo, lonely=lonely)
            if outofplace and it + 1 < repeat:
                (s_t, s_p), (r_t, r_p) = (r_t, r_p), (s_t, s_p)
        return from_dev(r_t, x.dtype, n)

    if os.environ.get("FTAR_LOOPBACK_MODE") == "capture":
        capture(comm, res, world, rank)
        return finish(comm, res)
    if os.environ.get("FTAR_LOOPBACK_MODE") == "ddp":
        ddp(comm, res, world, rank)
        return finish(comm, res)
    if os.environ.get("FTAR_LOOPBACK_MODE") == "full":
        full_size(comm, res, world, rank)
        return finish(comm, res)
    if os.environ.get("FTAR_LOOPBACK_MODE") == "first_contact":
        first_contact(comm, res, world, rank)
        return finish(comm, res)
    if os.environ.get("FTAR_LOOPBACK_MODE") == "write_race":
        write_race(comm, res, world, rank)
        return finish(comm, res)
    if os.environ.get("FTAR_LOOPBACK_MODE") == "soak":
        soak(comm, res, world, rank, run, int(os.environ.get("FTAR_LOOPBACK_SOAK", "40")))
        return finish(comm, res)

    forms = os.environ.get("FTAR_LOOPBACK_FORMS", "direct,stages,collective").split(",")
    for ag in forms:
        comm.allgather = ag
        comm.reduce_scatter = "stages" if ag == "stages" else "direct"
        for c in gc.allreduce_cases(max_n=max_n, filt=lambda c: c["P"] == world):
            x = gc.case_inputs(c)[rank]
            try:
                out = run(x, c["topo"], c["lonely"], c["dtype"], c["op"], c["outofplace"], c["repeat"])
                gc.check_output(c, rank, out)
                res["golden"] += 1
            except Exception as e:  # noqa: BLE001  reported per case
                res["fail"].append(f"{ag} {c['id']}: {str(e)[:300]}")

    comm.allgather, comm.reduce_scatter = "direct", "direct"
    n = (1 << 20) + 13
    for topo, dt, host in (("1", "f32", False), (str(world), "f32", False), ("1", "f32", True),
                           (str(world), "bf16", False)):
        ins = [fi.fill(dt, 77, r, n) for r in range(world)]
        try:
            out = run(ins[rank], topo, 0, fi.BY_NAME[dt], 0, True, host=host)
            ref = oracle_lib.allreduce(ins, topo, 0, dtype=fi.BY_NAME[dt])[rank]
            np.testing.assert_array_equal(out.view(np.uint8), ref.view(np.uint8))
            res["oracle"] += 1
        except Exception as e:  # noqa: BLE001
            res["fail"].append(f"oracle topo={topo} {dt} host={host}: {str(e)[:300]}")

    # RCCL's own collective on the same communicator (yardstick path of bench.py)
    try:
        x = fi.fill("i32", 5, rank, 4099)
        s_t, s_p = to_dev(x)
        r_t, r_p = filled_dev(x.nbytes)
        comm.rccl_allreduce(s_p, r_p, x.size, fi.BY_NAME["i32"], 0)
        want = np.sum([fi.fill("i32", 5, r, 4099).astype(np.int64) for r in range(world)], axis=0)
        np.testing.assert_array_equal(from_dev(r_t, np.int32, x.size), want.astype(np.int32))
        res["nccl_allreduce"] = "ok"
    except Exception as e:  # noqa: BLE001
        res["fail"].append(f"ncclAllReduce: {str(e)[:300]}")

    return finish(comm, res)


def write_result(res):
    """one file per rank (FTAR_LOOPBACK_OUT): ranks share stdout, where their lines can interleave"""
    d = os.environ.get("FTAR_LOOPBACK_OUT")
    if d:
        with open(os.path.join(d, f"rank{res['rank']}.json"), "w") as f:
            json.dump(res, f)


def finish(comm, res):
    import torch
    import torch.distributed as dist
    if "first_call" not in res:   # a broken communicator's stream may hold an aborted all-gather: not waited on
        torch.cuda.synchronize()
    comm.destroy()
    print("LOOPBACK " + json.dumps(res), flush=True)
    write_result(res)
    dist.barrier()
    dist.destroy_process_group()
    return 0 if not res["fail"] else 1


def soak(comm, res, world, rank, run, count):
    """Seeded random cases of this world size (tests/random_cases.py: ring, trees, lonely layouts, every dtype,
    SUM and BAND, ragged sizes down to 0 and 1 element, in place or out of place) over RCCL, each with a random
    pipeline piece size, data-movement form (direct, stages, collective, peer read / write, auto) and device,
    pinned-host or pageable-host buffers; every rank against the oracle.
    Every rank draws the same sequence, so the per-call settings agree across ranks."""
    import random

    import ftar_inputs as fi
    import random_cases
    rng = random.Random(4242 + world)
    res["soak"] = 0
    for c in random_cases.cases(seed=900 + world, count=count, P_fixed=world):
        # every data-movement form: the peer forms map the other processes' exchange buffers over IPC (plans
        # they cannot run, and host buffers, take the p2p path); "auto" takes the execution model's choice
        form = rng.choice(["direct", "stages", "collective", "peer-read", "peer-write", "auto"])
        chunk = rng.choice([0, 256, 4096, 1 << 16])
        host = rng.random() < 0.4
        pinned = rng.random() < 0.7
        try:
            comm.form = form
            comm.chunk_bytes = chunk
            comm.host_chunk_bytes = chunk
            out = run(c["ins"][rank], c["topo"], c["lonely"], fi.BY_NAME[c["dtype"]],
                      0 if c["op"] == "sum" else 1, c["oop"], host=host, pinned=pinned)
            if out.tobytes() != c["ref"][rank].tobytes():
                raise AssertionError("differs from the oracle")
            res["soak"] += 1
        except Exception as e:  # noqa: BLE001
            res["fail"].append(f"soak P={world} topo={c['topo']}+{c['lonely']} n={c['n']} {c['dtype']} "
                               f"{c['op']} oop={c['oop']} {form} chunk={chunk} host={host} pinned={pinned}: "
                               f"{str(e)[:200]}")
            return


def ddp(comm, res, world, rank):
    """DistributedDataParallel with ftar as its gradient AllReduce (ftar.ddp.allreduce_hook) against DDP's own
    gloo AllReduce: the same model, the same per-rank batches, 3 SGD steps, small buckets (several per step).
    At P = 2 the gradients are bit-identical (one rounded add either way, / 2 exact; in bf16 too: ftar adds in
    fp32 and rounds once, a bf16 add rounds its exact sum once); at P = 4 the two sum in different orders, so
    they agree to a relative 1e-5 (fp32) or 2e-2 (bf16) of each tensor's largest gradient."""
    import copy

    import torch
    import torch.distributed as dist
    from torch.nn.parallel import DistributedDataParallel as DDP

    import ftar.ddp
    torch.manual_seed(1234)
    dt = {"f32": torch.float32, "bf16": torch.bfloat16}[os.environ.get("FTAR_LOOPBACK_DDP_DTYPE", "f32")]
    net = torch.nn.Sequential(torch.nn.Linear(256, 1024), torch.nn.ReLU(), torch.nn.Linear(1024, 1000),
                              torch.nn.ReLU(), torch.nn.Linear(1000, 10)).cuda().to(dt)
    a = DDP(copy.deepcopy(net), device_ids=[0], bucket_cap_mb=1)
    b = DDP(copy.deepcopy(net), device_ids=[0], bucket_cap_mb=1)
    state = ftar.ddp.HookState(comm)
    a.register_comm_hook(state, ftar.ddp.allreduce_hook)
    oa = torch.optim.SGD(a.parameters(), lr=0.05)
    ob = torch.optim.SGD(b.parameters(), lr=0.05)
    g = torch.Generator(device="cuda")
    g.manual_seed(99 + rank)
    worst = 0.0
    for step in range(3):
        x = torch.randn(64, 256, device="cuda", generator=g).to(dt)
        y = torch.randint(0, 10, (64,), device="cuda", generator=g)
        for m, o in ((a, oa), (b, ob)):
            o.zero_grad()
            torch.nn.functional.cross_entropy(m(x), y).backward()
        torch.cuda.synchronize()
        for pa, pb in zip(a.parameters(), b.parameters()):
            if world == 2:   # a + b is one rounding either way, and / 2 is exact: identical bits
                if not torch.equal(pa.grad, pb.grad):
                    res["fail"].append(f"ddp step {step}: gradient differs from DDP's own AllReduce")
                    return
            else:
                d = (pa.grad.float() - pb.grad.float()).abs().max() / pb.grad.float().abs().max().clamp_min(1e-30)
                worst = max(worst, d.item())
        oa.step()
        ob.step()
        with torch.no_grad():   # the next step compares gradients of the same parameters
            for pa, pb in zip(a.parameters(), b.parameters()):
                pb.copy_(pa)
    res["ddp_hook_calls"] = state.calls
    res["ddp_worst_rel"] = worst
    if world != 2 and worst > (1e-5 if dt == torch.float32 else 2e-2):
        res["fail"].append(f"ddp: gradients differ by {worst:.3g} (relative) from DDP's own AllReduce")
    # every rank ends with the same parameters
    flat = torch.cat([p.detach().reshape(-1) for p in a.parameters()])
    first = flat.clone()
    dist.broadcast(first, 0)
    if not torch.equal(first, flat):
        res["fail"].append("ddp: ranks' parameters differ after 3 steps")


def full_size(comm, res, world, rank):
    """BASELINE's full buckets over RCCL at P = world (8 for C4/C5): C4 = 2^28 fp32 on the ring (direct and
    the reference's staged rounds, default pieces and pieces of 24 MiB + 4 KiB that divide no block), C5 = 2^29
    bf16 on the width-P tree; out of place, device-resident, random inputs that differ per rank.  Every rank
    regenerates all P inputs from their seeds and compares its WHOLE output bit for bit with the reference's
    fold over the whole bucket (tests/whole_fold.py, pinned to the oracle by tests/test_whole_fold.py)."""
    import torch

    import whole_fold
    res["full"] = []
    odd = 24 * (1 << 20) + 4096
    cases = [((1 << 28), "f32", "1", "direct", 0), ((1 << 28), "f32", "1", "stages", 0),
             ((1 << 29), "bf16", str(world), "direct", 0)]
    if os.environ.get("FTAR_RUN_WIDE") == "1":   # pieces that divide no block (in-process at full size by default)
        cases[2:2] = [((1 << 28), "f32", "1", "direct", odd), ((1 << 28), "f32", "1", "stages", odd)]
    for n, dt, topo, form, chunk in cases:
        tdt = {"f32": torch.float32, "bf16": torch.bfloat16}[dt]
        comm.allgather = form
        comm.reduce_scatter = "stages" if form == "stages" else "direct"
        comm.chunk_bytes = chunk

        def gen(r):
            g = torch.Generator(device="cuda")
            g.manual_seed(2024 + r)
            return (torch.rand(n, generator=g, device="cuda") * 2 - 1).to(tdt)

        x = gen(rank)
        y = torch.empty_like(x)
        comm.allreduce(x, y, n, dt, "sum", topo_=topo, stream=torch.cuda.current_stream())
        torch.cuda.synchronize()
        xs = [x if r == rank else gen(r) for r in range(world)]
        exp = whole_fold.fold(xs, n, "ring" if topo == "1" else "tree")
        bad = whole_fold.first_mismatch(y, exp)
        what = f"{dt} n={n} topo={topo} {form} chunk={chunk or 'default'}"
        res["full"].append(f"{what}: " + ("ok (whole bucket)" if bad is None else
                                          f"MISMATCH in {bad[0]} elements, first at {bad[1]}"))
        if bad is not None:
            res["fail"].append(res["full"][-1])
        del x, y, xs, exp
        torch.cuda.empty_cache()
    comm.chunk_bytes = 0


def write_race(comm, res, world, rank):
    """The peer-write form's exchange buffer across consecutive calls: a tiny call (its final blocks land at
    the end of the slot area, final_at = P * slot) then a larger one whose slots cover that final area.  The
    last rank enqueues its copy-out of every call late (FTAR_DEBUG_PEER_LATE_US, as a slow host would), so its
    peers are already scattering the next call into its exchange buffer: the call must not return on any rank
    before every rank's copy-out is done.  Small-integer inputs, so every result is exact."""
    import numpy as np
    import torch
    res["write_race"] = 0
    comm.form = "peer-write"
    for it in range(4):
        for n, dt, tdt in ((9, "f64", torch.float64), (100_003, "f32", torch.float32)):
            x = (torch.arange(n, device="cuda", dtype=torch.int64) % 7 - 3 + rank + it).to(tdt)
            y = torch.full_like(x, 55)
            comm.allreduce(x, y, n, dt, "sum", topo_="1")
            torch.cuda.synchronize()
            want = sum((torch.arange(n, dtype=torch.int64) % 7 - 3 + r + it) for r in range(world)).to(tdt)
            got = y.cpu()
            if not torch.equal(got, want):
                bad = int((got != want).sum())
                res["fail"].append(f"write_race it={it} n={n} {dt}: {bad} elements differ, first "
                                   f"{int(np.flatnonzero((got != want).numpy())[0])}")
                continue   # keep making the calls: the peers would wait in them
            res["write_race"] += 1


def first_contact(comm, res, world, rank):
    """A peer that never makes its first call: rank 0's first call on the RCCL communicator would
    block in the settings all-gather; it runs on a helper thread with a deadline (FTAR_FIRST_CONTACT_TIMEOUT_S,
    4 s here), so the call fails with FTAR_ERR_TIMEOUT after about that long, every later call fails at once,
    and the communicator is destroyed (RCCL aborted) without a hang.  The other ranks never call; they
    destroy their communicators after rank 0 is done."""
    import time

    import torch
    import torch.distributed as dist

    import ftar
    if rank == 0:
        x = torch.ones(4096, device="cuda")
        t0 = time.time()
        try:
            comm.allreduce(x, x, x.numel(), "f32", "sum", topo_="1", stream=torch.cuda.current_stream())
            res["fail"].append("the first call returned although no peer took part")
        except ftar.FtarError as e:
            res["first_call"] = {"status": e.status, "s": round(time.time() - t0, 2), "error": str(e)[:300]}
            if e.status != 7 or not 3 <= time.time() - t0 <= 60:
                res["fail"].append(f"first call: {res['first_call']}")
        t1 = time.time()
        try:
            comm.allreduce(x, x, x.numel(), "f32", "sum", topo_="1", stream=torch.cuda.current_stream())
            res["fail"].append("the second call on a broken communicator returned")
        except ftar.FtarError as e:
            res["second_call"] = {"status": e.status, "s": round(time.time() - t1, 3)}
            if e.status != 7 or time.time() - t1 > 1:
                res["fail"].append(f"second call: {res['second_call']}")
    dist.barrier()


def capture(comm, res, world, rank):
    """The product's process model under stream capture at P > 1: one rank per process over an RCCL
    communicator, ftar_allreduce (ring and the width-P tree, direct and staged forms) captured with
    torch.cuda.graph and replayed on new inputs; every replay equals the oracle's fold of that replay's
    inputs.  ncclSend/ncclRecv are captured as graph nodes, as a training step's gradient AllReduce would be."""
    import numpy as np
    import torch

    import ftar_inputs as fi
    import oracle_lib
    n = (1 << 18) + 7
    res["captured"] = 0
    for topo, ag in (("1", "direct"), (str(world), "direct"), ("1", "stages")):
        try:
            comm.allgather = ag
            comm.reduce_scatter = "stages" if ag == "stages" else "direct"
            x = torch.empty(n, device="cuda")
            y = torch.empty_like(x)
            x.copy_(torch.from_numpy(fi.fill("f32", 1, rank, n)))
            comm.allreduce(x, y, n, "f32", "sum", topo_=topo, stream=torch.cuda.current_stream())   # warm-up
            torch.cuda.synchronize()
            s0 = torch.cuda.Stream()
            g = torch.cuda.CUDAGraph()
            sys.stderr.write(f"[rank {rank}] capture topo={topo} {ag}: begin\n")
            with torch.cuda.graph(g, stream=s0,
                                  capture_error_mode=os.environ.get("FTAR_LOOPBACK_CAPTURE_MODE", "global")):
                comm.allreduce(x, y, n, "f32", "sum", topo_=topo, stream=s0)
            sys.stderr.write(f"[rank {rank}] capture topo={topo} {ag}: captured\n")
            for it in range(3):
                ins = [fi.fill("f32", 100 + it, r, n) for r in range(world)]
                x.copy_(torch.from_numpy(ins[rank]))
                y.zero_()
                torch.cuda.synchronize()
                g.replay()
                torch.cuda.synchronize()
                ref = oracle_lib.allreduce(ins, topo)[rank]
                np.testing.assert_array_equal(y.cpu().numpy().view(np.uint32), ref.view(np.uint32))
            del g
            res["captured"] += 1
        except Exception as e:  # noqa: BLE001
            res["fail"].append(f"capture topo={topo} {ag}: {str(e)[:300]}")


if __name__ == "__main__":
    try:
        sys.exit(main())
    except Exception:  # noqa: BLE001
        traceback.print_exc()
        err = {"rank": int(os.environ.get("RANK", -1)), "error": traceback.format_exc()[-1500:]}
        print("LOOPBACK " + json.dumps(err), flush=True)
        write_result(err)
        sys.exit(1)
