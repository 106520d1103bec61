#!/usr/bin/env python3
"""Peer-direct forms across P processes sharing one GPU (ftar_comm_init_host over gloo), at growing
bucket sizes, every call printed before and after -- a hang names the step it is in.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/peer_rehearsal.py \
        [--sizes 20,24,26,28] [--modes read,write,read-reg,write-reg]

faulthandler dumps every thread's Python stack after --stall seconds without progress and exits.
"""
import argparse
import faulthandler
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "allreduce-over-mpi_amd"), os.path.join(ROOT, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="20,24,26,28", help="log2 elements per rank (or =N elements), in call order")
    ap.add_argument("--modes", default="read,write,read-reg,write-reg")
    ap.add_argument("--topo", default=None)
    ap.add_argument("--stall", type=float, default=60.0)
    a = ap.parse_args()

    import torch
    import torch.distributed as dist

    import ftar
    import ftar.dist

    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = int(os.environ.get("LOCAL_RANK", rank)) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    t0 = time.time()

    def say(msg):
        faulthandler.dump_traceback_later(a.stall, exit=True)   # re-armed at every step
        sys.stderr.write(f"[rank {rank} {time.time() - t0:7.2f}s] {msg}\n")
        sys.stderr.flush()

    say("init_host_comm")
    comm = ftar.dist.init_host_comm(device=dev)
    topo = a.topo or ("1" if world > 1 else None)
    ok_all = True
    for tok in a.sizes.split(","):   # log2 of the element count, or =N for N elements
        n = int(tok[1:]) if tok.startswith("=") else 1 << int(tok)
        lg = tok
        x = torch.full((n,), float(rank + 1), device="cuda")
        for mode in a.modes.split(","):
            reg = mode.endswith("-reg")
            xin, y = (x.clone(), torch.empty_like(x))
            ids = []
            if reg:
                say(f"2^{lg} register")
                try:
                    ids = [comm.register(xin, n * 4)]
                    ids.append(comm.register(y, n * 4))
                except ftar.FtarError as e:   # refused on every rank alike (e.g. FTAR_IPC_SIZE_GUARD)
                    say(f"2^{lg} {mode}: registration refused ({e}); skipped")
                    for i in ids:
                        comm.deregister(i)
                    dist.barrier()
                    continue
            comm.peer_direct = mode.split("-")[0]
            for it in range(3):
                say(f"2^{lg} {mode} call {it}")
                comm.allreduce(xin, y, n, "f32", "sum", topo_=topo)
                torch.cuda.synchronize()
            exp = float(world * (world + 1) // 2)
            ok = bool((y == exp).all())
            ok_all &= ok
            say(f"2^{lg} {mode} {'ok' if ok else 'MISMATCH'}")
            for i in ids:
                comm.deregister(i)
            del xin, y
            dist.barrier()
    say("destroy")
    comm.destroy()
    dist.destroy_process_group()
    faulthandler.cancel_dump_traceback_later()
    if rank == 0:
        print("peer rehearsal", "ok" if ok_all else "MISMATCH", flush=True)
    sys.exit(0 if ok_all else 1)


if __name__ == "__main__":
    main()
