"""ftar as the gradient AllReduce of torch DistributedDataParallel (a DDP communication hook).

The data-parallel caller of the hot path: DDP packs gradients into buckets and hands each bucket to a hook
once its gradients are ready; the hook below reduces the bucket in place with ftar_allreduce on the stream the
backward pass runs on (the FlexTree schedule of FT_TOPO / FT_LONELY or `topo`, else the cost model; RCCL p2p
over xGMI, the reduce kernel on ftar's own stream); the bucket is divided by the world size first, as DDP's own
allreduce hook does (so the mean rounds as DDP's does and keeps its overflow headroom).  No host
synchronisation: the AllReduce and every later use of the bucket are ordered after the division by that
stream.

    comm = ftar.dist.init_comm()                       # one rank per GPU, RCCL over the DDP process group's ids
    model = DistributedDataParallel(model, device_ids=[local_rank])
    model.register_comm_hook(ftar.ddp.HookState(comm), ftar.ddp.allreduce_hook)

The reference reduces MPI buffers (MPI_Allreduce_FT, mpi_mod.hpp:1723-1778); a DDP bucket is the same call on
a device tensor, in place (`sendbuf = MPI_IN_PLACE`).
"""
import torch

import ftar


class HookState:
    """What the hook needs: the ftar communicator, and optionally a fixed topology (FT_TOPO syntax)."""

    def __init__(self, comm, topo=None, lonely=0):
        self.comm, self.topo, self.lonely = comm, topo, lonely
        self.calls = 0


def allreduce_hook(state, bucket):
    """DDP comm hook: the bucket / world size (first, as torch's default hook divides before it reduces), then
    its in-place FlexTree AllReduce; returns a completed future whose tensor the reducer copies back into the
    gradients on the same stream."""
    t = bucket.buffer()
    stream = torch.cuda.current_stream(t.device)
    t.div_(state.comm.nranks)
    state.comm.allreduce(None, t, t.numel(), ftar._dt(str(t.dtype)), "sum", topo_=state.topo, lonely=state.lonely,
                         stream=stream)
    state.calls += 1
    fut = torch.futures.Future(devices=[t.device])
    fut.set_result(t)
    return fut
