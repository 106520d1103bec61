#!/usr/bin/env python3
"""Host-buffer AllReduce on the host-bootstrapped communicator (the MPI drop-in's `ipc` transport):
piece-pipelined read form (peer_allreduce_host) against the whole-bucket path, same run, interleaved.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/host_ipc_rate.py \
        [--sizes 24,26,28] [--iters 5] [--pieces 0,4194304]

Prints one JSON line per (size, path) on rank 0: min and median ms over --iters calls, algBW per rank.
Ranks on one GPU share its one PCIe link, so these are not per-rank link rates of a node.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "allreduce-over-mpi_amd"), os.path.join(ROOT, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="24,26,28", help="log2 fp32 elements per rank")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--pieces", default="0", help="host piece bytes for the pipelined path (0 = auto)")
    ap.add_argument("--topo", default="1")
    ap.add_argument("--inplace", action="store_true", help="MPI_IN_PLACE, as the reference harness calls it")
    ap.add_argument("--register", action="store_true", help="hipHostRegister'ed numpy buffers (the MPI drop-in's "
                    "MPI_Allreduce_FT_register) instead of torch pinned allocations")
    a = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    import ftar
    import ftar.dist

    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = int(os.environ.get("LOCAL_RANK", rank)) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    comms = {}
    for name, env in (("pipelined", "1"), ("whole", "0")):
        os.environ["FTAR_HOST_PEER_PIPELINE"] = env
        comms[name] = ftar.dist.init_host_comm(device=dev)
        comms[name].peer_direct = "read"
    for tok in a.sizes.split(","):
        n = 1 << int(tok)
        if a.register:
            import ctypes
            hip = ctypes.CDLL("libamdhip64.so")
            x, y = np.empty(n, np.float32), np.empty(n, np.float32)
            for b in (x, y):
                rc = hip.hipHostRegister(ctypes.c_void_p(b.ctypes.data), ctypes.c_size_t(b.nbytes), ctypes.c_uint(0))
                assert rc == 0, rc
        else:
            x = torch.empty(n, dtype=torch.float32, pin_memory=True).numpy()
            y = torch.empty(n, dtype=torch.float32, pin_memory=True).numpy()
        x[:] = np.float32(rank + 1)
        want = np.float32(world * (world + 1) // 2)
        configs = [("whole", 0)] + [("pipelined", int(p)) for p in a.pieces.split(",")]
        times = {c: [] for c in configs}
        for it in range(a.iters + 1):
            for name, piece in configs:
                c = comms[name]
                c.host_chunk_bytes = piece
                dist.barrier()
                t0 = time.perf_counter()
                if a.inplace:
                    c.allreduce_host(None, x, n, "f32", "sum", topo_=a.topo)
                else:
                    c.allreduce_host(x, y, n, "f32", "sum", topo_=a.topo)
                torch.cuda.synchronize()
                t = time.perf_counter() - t0
                out = x if a.inplace else y
                ok = bool((out[:: max(1, n // 4096)] == want).all() and out[-1] == want)
                if a.inplace:
                    x[:] = np.float32(rank + 1)
                tt = torch.tensor([t, 0.0 if ok else 1.0], dtype=torch.float64)
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                if tt[1] > 0:
                    raise SystemExit(f"wrong result: {name} piece {piece} 2^{tok}")
                if it:  # the first call maps the exchange buffers
                    times[(name, piece)].append(float(tt[0]))
                y[:] = 0
        if rank == 0:
            for (name, piece), ts in times.items():
                ts.sort()
                print(json.dumps({"elements": n, "bytes_per_rank": n * 4, "ranks": world, "path": name,
                                  "piece_bytes": piece, "ms_min": round(ts[0] * 1e3, 3),
                                  "ms_med": round(ts[len(ts) // 2] * 1e3, 3),
                                  "algbw_GBps_min_time": round(n * 4 / ts[0] / 1e9, 2)}), flush=True)
    for c in comms.values():
        c.destroy()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
