/*
 * ftar_mpi.h — the reference's call surface, MPI flavoured (libftar_mpi.so).
 *
 * Drop-in for the FlexTree entry point of DictXiong/AllReduce-Over-MPI:
 *
 *   int MPI_Allreduce_FT(const void *sendbuf, void *recvbuf, int count,
 *                        MPI_Datatype datatype, MPI_Op op, MPI_Comm comm)
 *     — allreduce_over_mpi/mpi_mod.hpp:1724 (STANDALONE_TEST build); in the
 *       plugin build the same body is a file-static MPI_Allreduce (:1726).
 *
 * Same arguments and semantics: host buffers (the MPI send/recv buffers of
 * the caller), sendbuf == MPI_IN_PLACE reduces recvbuf in place, collective
 * over `comm`, FT_TOPO / FT_LONELY read from the environment on EVERY call as
 * get_stages is (mpi_mod.hpp:1732; both unset: the re-fitted cost model
 * instead of the reference's exit(1); set but invalid for the communicator's
 * size: MPI_ERR_ARG on every rank before anything moves, 1-rank calls
 * included, where the reference prints "invalid FT_TOPO" and exit(1)s,
 * :1471-1475).  Underneath:
 * one GPU per rank (node-local rank % visible devices, or FTAR_DEVICE),
 * H2D -> device AllReduce (RCCL p2p over xGMI + HIP reduce kernel) -> D2H.
 * FTAR_MPI_TRANSPORT=auto (default) | rccl | ipc: ipc bootstraps over `comm`
 * itself (MPI_Allgather) and moves blocks with kernel loads through
 * IPC-mapped buffers, no RCCL; auto takes it on every rank when RCCL cannot
 * initialise on some rank (e.g. ranks sharing a GPU).
 * Results are bit-identical to the reference for the same FT_TOPO.
 *
 * Errors: the reference always returns 0 and exit(1)s on bad input
 * (mpi_mod.hpp:1321, :1384, :1405, :1474); this returns MPI_ERR_TYPE /
 * MPI_ERR_OP / MPI_ERR_ARG / MPI_ERR_OTHER instead.
 */
#ifndef FTAR_MPI_H
#define FTAR_MPI_H

#include <mpi.h>

#include "ftar.h"

#ifdef __cplusplus
extern "C" {
#endif

int MPI_Allreduce_FT(const void* sendbuf, void* recvbuf, int count, MPI_Datatype datatype, MPI_Op op, MPI_Comm comm);

/* Same collective on DEVICE buffers (no host staging), enqueued on `stream`
 * (hipStream_t; NULL = the communicator's internal stream, synchronised). */
int MPI_Allreduce_FT_device(const void* sendbuf, void* recvbuf, int count, MPI_Datatype datatype, MPI_Op op,
                            MPI_Comm comm, void* stream);

/* The ftar communicator bound to an MPI communicator (created on first use). */
int MPI_Allreduce_FT_comm(MPI_Comm comm, ftar_comm_t* out);

/* Pin a host buffer for the copies of MPI_Allreduce_FT (hipHostRegister),
 * until MPI_Allreduce_FT_unregister; the caller keeps it alive meanwhile.
 * Calls on unregistered buffers copy pageable, unless FTAR_MPI_REGISTER=1
 * (pin every buffer passed in, at most FTAR_MPI_REGISTER_MAX = 4 kept, least
 * recently used evicted: the caller must not free such a buffer while it may
 * be cached).  unregister returns MPI_ERR_ARG for an unknown pointer and
 * MPI_ERR_PENDING while a call copies through it. */
int MPI_Allreduce_FT_register(const void* buf, size_t bytes);
int MPI_Allreduce_FT_unregister(const void* buf);

/* Release every cached communicator, device buffer and host registration.
 * Optional: each communicator's state is also released by MPI_Comm_free (an
 * MPI attribute with a delete callback; MPI_Finalize for MPI_COMM_WORLD), and
 * a communicator created later under the same handle starts fresh.  (The
 * reference leaks its buffer, mpi_mod.hpp:1489, and a communicator per call,
 * :1541-1548.) */
int MPI_Allreduce_FT_finalize(void);

/* Map an MPI datatype / op of the reference (mpi_mod.hpp:1363-1412) to ftar. */
int ftar_mpi_dtype(MPI_Datatype datatype, ftar_dtype_t* out);
int ftar_mpi_op(MPI_Op op, ftar_op_t* out);

#ifdef __cplusplus
}
#endif
#endif /* FTAR_MPI_H */
