"""Bring-up of an ftar communicator inside a torch.distributed job.

One process per GPU (torchrun): rank 0 creates the RCCL unique id, every rank
receives it over the already-initialised torch.distributed process group
(any backend, gloo is enough), then ftar_comm_init_rank builds the RCCL
communicator on this rank's device.  This replaces the MPI_Comm the reference
runs on (MPI_Comm_size/rank, mpi_mod.hpp:781-809).
"""
import os

import ftar


def exchange_unique_id(group=None):
    import torch.distributed as dist
    obj = [ftar.get_unique_id() if dist.get_rank(group) == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    return obj[0]


def init_comm(device=None, group=None):
    """ftar.Comm for this rank; device defaults to LOCAL_RANK."""
    import torch.distributed as dist
    if device is None:
        device = int(os.environ.get("LOCAL_RANK", dist.get_rank(group)))
    uid = exchange_unique_id(group)
    return ftar.Comm.init_rank(dist.get_world_size(group), uid, dist.get_rank(group), device)


def init_host_comm(device=None, group=None):
    """ftar.Comm bootstrapped over the torch.distributed group itself (no RCCL; ftar_comm_init_host):
    the peer-direct forms only.  Ranks may share a device."""
    import torch
    import torch.distributed as dist
    if device is None:
        device = int(os.environ.get("LOCAL_RANK", dist.get_rank(group)))
    world = dist.get_world_size(group)

    def allgather(mine):
        t = torch.frombuffer(bytearray(mine), dtype=torch.uint8)
        outs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(outs, t, group=group)
        return [o.numpy().tobytes() for o in outs]
    return ftar.Comm.init_host(world, dist.get_rank(group), device, allgather)
