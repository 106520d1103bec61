// MPI_Allreduce_FT on MI355X: the reference's host-buffer entry point
// (allreduce_over_mpi/mpi_mod.hpp:1723-1778) re-expressed over libftar.
//
//   reference                               here
//   get_stages() every call (:1732)         FT_TOPO/FT_LONELY read once per communicator
//   FlexTree_Context (:1734)                ftar plan cache (per topology, count)
//   P <= 1 -> memcpy (:1739-1746)           same, on the host
//   static grow-only host recv_buffer       grow-only DEVICE staging buffer per communicator
//   (:1489-1507, never freed)               (freed by MPI_Allreduce_FT_finalize)
//   ring/tree over MPI_Isend/Irecv          ftar_allreduce_host: H2D, RCCL p2p + HIP reduce and
//   + 14-thread OpenMP reduce               D2H pipelined piece by piece (PCIe in and out overlap)
//   MPI_Comm_split every call, leaked       nothing per call; RCCL comm built once
//   (:1541-1548)                            (or, FTAR_MPI_TRANSPORT=ipc / RCCL failing, a
//                                           communicator bootstrapped over MPI: peer forms)
// The caller's buffers are page-locked on first use (hipHostRegister, cached)
// so the copies run at PCIe DMA speed; set FTAR_MPI_REGISTER=0 to disable.
#include <hip/hip_runtime_api.h>

#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <utility>

#include "ftar_mpi.h"

namespace {

struct Entry {
  ftar_comm_t comm = nullptr;
  int rank = 0, size = 1, device = 0;
  hipStream_t stream = nullptr;
  MPI_Comm boot = MPI_COMM_NULL;  // ipc transport: the duplicate the communicator bootstraps over
  bool ipc = false;
};

std::mutex g_mu;
std::map<MPI_Comm, Entry> g_entries;
std::map<void*, size_t> g_registered;

int pick_device(MPI_Comm comm) {
  if (const char* e = getenv("FTAR_DEVICE")) return atoi(e);
  MPI_Comm node;
  int local = 0;
  if (MPI_Comm_split_type(comm, MPI_COMM_TYPE_SHARED, 0, MPI_INFO_NULL, &node) == MPI_SUCCESS) {
    MPI_Comm_rank(node, &local);
    MPI_Comm_free(&node);
  }
  int n = 1;
  if (hipGetDeviceCount(&n) != hipSuccess || n < 1) n = 1;
  return local % n;
}

// the host collective of an ipc-transport communicator (ftar_comm_init_host)
int mpi_allgather(const void* mine, void* all, size_t bytes, void* user) {
  MPI_Comm c = *static_cast<MPI_Comm*>(user);
  return MPI_Allgather(mine, (int)bytes, MPI_BYTE, all, (int)bytes, MPI_BYTE, c) == MPI_SUCCESS ? 0 : 1;
}

// FTAR_MPI_TRANSPORT: rccl (RCCL p2p, every form), ipc (a communicator
// bootstrapped over MPI itself: the peer-direct read form over IPC-mapped
// buffers, no RCCL), auto (default: RCCL, and ipc on every rank when the RCCL
// communicator fails to come up on any rank -- e.g. ranks sharing a GPU)
int entry_for(MPI_Comm comm, Entry** out) {
  auto it = g_entries.find(comm);
  if (it != g_entries.end()) {
    *out = &it->second;
    return MPI_SUCCESS;
  }
  Entry& e = g_entries.emplace(comm, Entry{}).first->second;  // stable address: `boot` is the callback's state
  auto fail = [&](int rc) {
    if (e.boot != MPI_COMM_NULL) MPI_Comm_free(&e.boot);
    g_entries.erase(comm);
    return rc;
  };
  MPI_Comm_rank(comm, &e.rank);
  MPI_Comm_size(comm, &e.size);
  e.device = pick_device(comm);
  if (e.size > 1) {
    const char* m = getenv("FTAR_MPI_TRANSPORT");
    const std::string mode = m && *m ? m : "auto";
    if (mode != "rccl" && mode != "ipc" && mode != "auto") return fail(MPI_ERR_ARG);
    int rccl_ok = 0;
    if (mode != "ipc") {
      ftar_unique_id_t id;
      memset(&id, 0, sizeof id);
      int ok = e.rank == 0 ? ftar_get_unique_id(&id) == FTAR_SUCCESS : 1;
      MPI_Bcast(&ok, 1, MPI_INT, 0, comm);
      if (ok) {
        MPI_Bcast(&id, (int)sizeof id, MPI_BYTE, 0, comm);
        rccl_ok = ftar_comm_init_rank(&e.comm, e.size, id, e.rank, e.device) == FTAR_SUCCESS;
      }
      int all_ok = rccl_ok;
      MPI_Allreduce(&rccl_ok, &all_ok, 1, MPI_INT, MPI_MIN, comm);  // every rank takes the same path
      if (!all_ok && e.comm) {
        ftar_comm_destroy(e.comm);
        e.comm = nullptr;
      }
      rccl_ok = all_ok;
      if (!rccl_ok && mode == "rccl") return fail(MPI_ERR_OTHER);
    }
    if (!rccl_ok) {
      if (MPI_Comm_dup(comm, &e.boot) != MPI_SUCCESS) return fail(MPI_ERR_OTHER);
      if (ftar_comm_init_host(&e.comm, e.size, e.rank, e.device, mpi_allgather, &e.boot) != FTAR_SUCCESS)
        return fail(MPI_ERR_OTHER);
      int pd = 0;
      if (ftar_comm_get_peer_direct(e.comm, &pd) == FTAR_SUCCESS && pd == 0)
        (void)ftar_comm_set_peer_direct(e.comm, FTAR_PEER_READ);
      e.ipc = true;
    }
  }
  *out = &e;
  return MPI_SUCCESS;
}

// device + stream on first GPU use (a 1-rank communicator's host path never needs them)
int ensure_stream(Entry* e) {
  if (hipSetDevice(e->device) != hipSuccess) return MPI_ERR_OTHER;
  if (!e->stream && hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) return MPI_ERR_OTHER;
  return MPI_SUCCESS;
}

void maybe_register(const void* p, size_t bytes) {
  static const bool on = !getenv("FTAR_MPI_REGISTER") || atoi(getenv("FTAR_MPI_REGISTER")) != 0;
  if (!on || !p || !bytes) return;
  void* key = const_cast<void*>(p);
  auto it = g_registered.find(key);
  if (it != g_registered.end() && it->second >= bytes) return;
  if (it != g_registered.end()) {
    (void)hipHostUnregister(key);
    g_registered.erase(it);
  }
  if (hipHostRegister(key, bytes, hipHostRegisterDefault) == hipSuccess) g_registered[key] = bytes;
  else (void)hipGetLastError();  // pageable copies still work
}

}  // namespace

extern "C" {

int ftar_mpi_dtype(MPI_Datatype d, ftar_dtype_t* out) {
  // handle_reduce's dispatch list, mpi_mod.hpp:1365-1375
  if (d == MPI_UINT8_T) *out = FTAR_UINT8;
  else if (d == MPI_INT8_T) *out = FTAR_INT8;
  else if (d == MPI_UINT16_T) *out = FTAR_UINT16;
  else if (d == MPI_INT16_T) *out = FTAR_INT16;
  else if (d == MPI_INT32_T) *out = FTAR_INT32;
  else if (d == MPI_INT64_T || d == MPI_LONG_LONG_INT || d == MPI_LONG_LONG) *out = FTAR_INT64;
  else if (d == MPI_FLOAT) *out = FTAR_FLOAT32;
  else if (d == MPI_DOUBLE) *out = FTAR_FLOAT64;
  else if (d == MPI_C_BOOL) *out = FTAR_BOOL;
  else return MPI_ERR_TYPE;
  return MPI_SUCCESS;
}

int ftar_mpi_op(MPI_Op op, ftar_op_t* out) {
  if (op == MPI_SUM) *out = FTAR_SUM;
  else if (op == MPI_BAND) *out = FTAR_BAND;
  else return MPI_ERR_OP;
  return MPI_SUCCESS;
}

int MPI_Allreduce_FT_comm(MPI_Comm comm, ftar_comm_t* out) {
  std::lock_guard<std::mutex> g(g_mu);
  Entry* e;
  int rc = entry_for(comm, &e);
  if (rc == MPI_SUCCESS) *out = e->comm;
  return rc;
}

int MPI_Allreduce_FT(const void* sendbuf, void* recvbuf, int count, MPI_Datatype datatype, MPI_Op op,
                     MPI_Comm comm) {
  ftar_dtype_t dt;
  ftar_op_t fo;
  if (ftar_mpi_dtype(datatype, &dt) != MPI_SUCCESS) return MPI_ERR_TYPE;
  if (ftar_mpi_op(op, &fo) != MPI_SUCCESS) return MPI_ERR_OP;
  if (count < 0 || (!recvbuf && count)) return MPI_ERR_ARG;
  std::lock_guard<std::mutex> g(g_mu);
  Entry* e;
  int rc = entry_for(comm, &e);
  if (rc != MPI_SUCCESS) return rc;
  const size_t bytes = (size_t)count * ftar_dtype_size(dt);
  const void* src = sendbuf == MPI_IN_PLACE ? recvbuf : sendbuf;
  if (e->size <= 1) {  // mpi_mod.hpp:1739-1746
    if (src != recvbuf && bytes) memcpy(recvbuf, src, bytes);
    return MPI_SUCCESS;
  }
  if ((rc = ensure_stream(e)) != MPI_SUCCESS) return rc;
  maybe_register(src, bytes);
  maybe_register(recvbuf, bytes);
  const ftar_status_t st = ftar_allreduce_host(src == recvbuf ? nullptr : src, recvbuf, (size_t)count, dt, fo,
                                               nullptr, e->comm, e->stream);
  if (st == FTAR_ERR_HIP && hipGetLastError() == hipErrorOutOfMemory) return MPI_ERR_NO_MEM;
  if (st != FTAR_SUCCESS) return MPI_ERR_OTHER;
  if (hipStreamSynchronize(e->stream) != hipSuccess) return MPI_ERR_OTHER;
  return MPI_SUCCESS;
}

int MPI_Allreduce_FT_device(const void* sendbuf, void* recvbuf, int count, MPI_Datatype datatype, MPI_Op op,
                            MPI_Comm comm, void* stream) {
  ftar_dtype_t dt;
  ftar_op_t fo;
  if (ftar_mpi_dtype(datatype, &dt) != MPI_SUCCESS) return MPI_ERR_TYPE;
  if (ftar_mpi_op(op, &fo) != MPI_SUCCESS) return MPI_ERR_OP;
  if (count < 0) return MPI_ERR_ARG;
  std::lock_guard<std::mutex> g(g_mu);
  Entry* e;
  int rc = entry_for(comm, &e);
  if (rc != MPI_SUCCESS) return rc;
  if ((rc = ensure_stream(e)) != MPI_SUCCESS) return rc;
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : e->stream;
  const void* src = sendbuf == MPI_IN_PLACE ? nullptr : sendbuf;
  if (e->size <= 1) {
    if (src && src != recvbuf && count &&
        hipMemcpyAsync(recvbuf, src, (size_t)count * ftar_dtype_size(dt), hipMemcpyDeviceToDevice, s) != hipSuccess)
      return MPI_ERR_OTHER;
  } else if (ftar_allreduce(src, recvbuf, (size_t)count, dt, fo, nullptr, e->comm, s) != FTAR_SUCCESS) {
    return MPI_ERR_OTHER;
  }
  if (!stream && hipStreamSynchronize(s) != hipSuccess) return MPI_ERR_OTHER;
  return MPI_SUCCESS;
}

int MPI_Allreduce_FT_finalize(void) {
  std::lock_guard<std::mutex> g(g_mu);
  for (auto& kv : g_entries) {
    Entry& e = kv.second;
    (void)hipSetDevice(e.device);
    if (e.stream) (void)hipStreamSynchronize(e.stream);
    if (e.comm) ftar_comm_destroy(e.comm);
    if (e.stream) (void)hipStreamDestroy(e.stream);
    if (e.boot != MPI_COMM_NULL) MPI_Comm_free(&e.boot);
  }
  g_entries.clear();
  for (auto& kv : g_registered) (void)hipHostUnregister(kv.first);
  g_registered.clear();
  return MPI_SUCCESS;
}

}  // extern "C"
