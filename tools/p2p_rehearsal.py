#!/usr/bin/env python3
"""The engine's point-to-point forms across P processes sharing one GPU (host transport: bounce-buffer p2p
completed with host collectives), with exactly-summable inputs, so every element of the result is known:
x_r[i] = (i % 7) + r, y[i] = P * (i % 7) + P(P-1)/2.  Prints mismatch counts and the first bad indices.

    python -m torch.distributed.run --nproc-per-node 4 --master-addr 127.0.0.1 tools/p2p_rehearsal.py \
        [--configs "4:direct:direct:16777216;2,2:stages:stages:0"] [--log2n 28]
"""
import argparse
import faulthandler
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "allreduce-over-mpi_amd"), os.path.join(ROOT, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="4:direct:direct:16777216;4:direct:direct:1048576;2,2:direct:direct:16777216",
                    help="topology:reduce-scatter:all-gather:chunk bytes, ';'-separated")
    ap.add_argument("--log2n", type=int, default=28)
    ap.add_argument("--calls", type=int, default=3)
    ap.add_argument("--repeat", type=int, default=1, help="fresh communicator per repetition (buffers regrow)")
    ap.add_argument("--negate", action="store_true", help="alternate the sign of the inputs between calls")
    ap.add_argument("--stall", type=float, default=60.0, help="dump every thread's stack and exit after this long")
    a = ap.parse_args()
    os.environ["FTAR_HOST_P2P"] = "1"   # the experimental bounce-buffer p2p of the host transport
    import torch
    import torch.distributed as dist
    import ftar
    import ftar.dist
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    n = 1 << a.log2n
    i7 = (torch.arange(n, device="cuda", dtype=torch.int64) % 7).float()
    x = i7 + rank
    exp = i7 * world + world * (world - 1) // 2
    ok_all = True
    for rep in range(a.repeat):
        faulthandler.dump_traceback_later(a.stall, exit=True)
        comm = ftar.dist.init_host_comm(device=0)
        for cfg in a.configs.split(";"):
            topo, rs, ag, chunk = cfg.rsplit(":", 3)
            comm.reduce_scatter, comm.allgather, comm.chunk_bytes = rs, ag, int(chunk)
            for call in range(a.calls):
                sign = -1.0 if (a.negate and call % 2) else 1.0
                faulthandler.dump_traceback_later(a.stall, exit=True)
                y = torch.full_like(x, -1.0)
                comm.allreduce(x * sign, y, n, "f32", "sum", topo_=topo)
                torch.cuda.synchronize()
                bad = (y != exp * sign).nonzero().flatten()
                nb = int(bad.numel())
                cnt = torch.tensor([nb], dtype=torch.int64)
                dist.all_reduce(cnt)
                if nb:
                    lo, hi = int(bad[0]), int(bad[-1])
                    vals = [(int(i), float(y[i]), float(exp[i] * sign)) for i in bad[:3]]
                    print(f"[rank {rank}] rep {rep} {cfg} call {call}: {nb} bad in [{lo}, {hi}]; first {vals}",
                          flush=True)
                elif rank == 0 and call == a.calls - 1:
                    print(f"[rank 0] rep {rep} {cfg}: ok (all ranks {int(cnt)} bad)", flush=True)
                ok_all &= int(cnt) == 0
        faulthandler.dump_traceback_later(a.stall, exit=True)
        comm.destroy()
    faulthandler.cancel_dump_traceback_later()
    dist.destroy_process_group()
    if rank == 0:
        print("p2p rehearsal", "ok" if ok_all else "MISMATCH", flush=True)


if __name__ == "__main__":
    main()
