// MPI_Allreduce_FT on MI355X: the reference's host-buffer entry point
// (allreduce_over_mpi/mpi_mod.hpp:1723-1778) re-expressed over libftar.
//
//   reference                               here
//   get_stages() every call (:1732)         same: FT_TOPO/FT_LONELY read on every call; unset
//   invalid FT_TOPO -> exit(1) (:1471-1475)  -> cost model; set but invalid -> MPI_ERR_ARG on
//                                           every rank, before anything moves (P = 1 included)
//   FlexTree_Context (:1734)                ftar plan cache (per topology, count)
//   P <= 1 -> memcpy (:1739-1746)           same, on the host
//   static grow-only host recv_buffer       grow-only DEVICE staging buffer per communicator
//   (:1489-1507, never freed)               (freed with the communicator: MPI_Comm_free,
//                                           MPI_Finalize or MPI_Allreduce_FT_finalize)
//   ring/tree over MPI_Isend/Irecv          ftar_allreduce_host: H2D, RCCL p2p + HIP reduce and
//   + 14-thread OpenMP reduce               D2H pipelined piece by piece (PCIe in and out overlap)
//   MPI_Comm_split every call, leaked       nothing per call; RCCL comm built once
//   (:1541-1548)                            (or, FTAR_MPI_TRANSPORT=ipc / RCCL failing, a
//                                           communicator bootstrapped over MPI: peer forms)
// Host buffers: MPI_Allreduce_FT_register pins a buffer the caller owns until
// MPI_Allreduce_FT_unregister (like RCCL's user-buffer registration), so its
// copies run at PCIe DMA speed; FTAR_MPI_REGISTER=1 additionally pins every
// buffer passed in, keeping at most FTAR_MPI_REGISTER_MAX (default 4) such
// automatic registrations (least recently used evicted) -- the caller then
// promises not to free a buffer it passed while it may still be registered.
// Unregistered buffers take pageable copies.
//
// Communicators: the ftar state of an MPI communicator hangs on it as an MPI
// attribute (keyval with a delete callback), so MPI_Comm_free -- or
// MPI_Finalize for MPI_COMM_WORLD/SELF -- releases it, and a communicator
// created later under a recycled handle starts fresh.  Each has its own lock,
// held across its collectives; a process-wide lock only guards the keyval
// and the registrations, never a collective (MPI_THREAD_MULTIPLE callers on
// different communicators run concurrently, benchmark.cpp:50).
#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <utility>
#include <vector>

#include "ftar_mpi.h"

namespace {

struct Entry {
  std::mutex mu;  // one collective at a time on this communicator
  bool ready = false;
  ftar_comm_t comm = nullptr;
  int rank = 0, size = 1, device = 0;
  hipStream_t stream = nullptr;
  MPI_Comm owner = MPI_COMM_NULL;  // the communicator the attribute hangs on
  MPI_Comm boot = MPI_COMM_NULL;   // ipc transport: the duplicate the communicator bootstraps over
  bool ipc = false;
};

std::mutex g_mu;  // keyval, live set, registrations
int g_keyval = MPI_KEYVAL_INVALID;
std::set<Entry*> g_live;

struct Registration {
  size_t bytes = 0;
  bool automatic = false;  // FTAR_MPI_REGISTER=1 (evictable) vs MPI_Allreduce_FT_register
  int in_use = 0;          // calls copying through it right now (never evicted then)
  uint64_t last_use = 0;
};
std::map<uintptr_t, Registration> g_registered;
uint64_t g_tick = 0;

void release(Entry* e) {
  if (e->comm || e->stream) (void)hipSetDevice(e->device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  if (e->comm) ftar_comm_destroy(e->comm);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  if (e->boot != MPI_COMM_NULL) MPI_Comm_free(&e->boot);
  e->comm = nullptr;
  e->stream = nullptr;
  e->ready = false;
  e->ipc = false;
}

// MPI_Comm_free / MPI_Finalize / MPI_Comm_delete_attr of a communicator with ftar state
int delete_entry(MPI_Comm, int, void* val, void*) {
  Entry* e = static_cast<Entry*>(val);
  {
    std::lock_guard<std::mutex> g(g_mu);
    g_live.erase(e);
  }
  {
    std::lock_guard<std::mutex> g(e->mu);
    release(e);
  }
  delete e;
  return MPI_SUCCESS;
}

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

// The entry of `comm` (created empty on first sight).  Only the lookup holds
// the process-wide lock: bring-up is collective and runs under the entry's own
// lock (init_entry), so two threads bringing up two communicators in opposite
// orders on different ranks cannot deadlock on it.
int lookup(MPI_Comm comm, Entry** out) {
  if (comm == MPI_COMM_NULL) return MPI_ERR_COMM;
  std::lock_guard<std::mutex> g(g_mu);
  if (g_keyval == MPI_KEYVAL_INVALID &&
      MPI_Comm_create_keyval(MPI_COMM_NULL_COPY_FN, delete_entry, &g_keyval, nullptr) != MPI_SUCCESS)
    return MPI_ERR_OTHER;
  void* val = nullptr;
  int flag = 0;
  if (MPI_Comm_get_attr(comm, g_keyval, &val, &flag) != MPI_SUCCESS) return MPI_ERR_COMM;
  if (flag) {
    *out = static_cast<Entry*>(val);
    return MPI_SUCCESS;
  }
  Entry* e = new Entry;
  e->owner = comm;
  if (MPI_Comm_set_attr(comm, g_keyval, e) != MPI_SUCCESS) {
    delete e;
    return MPI_ERR_OTHER;
  }
  g_live.insert(e);
  *out = e;
  return MPI_SUCCESS;
}

// FTAR_MPI_TRANSPORT: rccl (RCCL p2p, every form), ipc (a communicator
// bootstrapped over MPI itself: the peer-direct read form over IPC-mapped
// buffers, no RCCL), auto (default: RCCL, and ipc on every rank when the RCCL
// communicator fails to come up on any rank -- e.g. ranks sharing a GPU).
// Called with e->mu held; a failed bring-up leaves the entry empty, and the
// next call tries again.
int init_entry(Entry* e, MPI_Comm comm) {
  if (e->ready) return MPI_SUCCESS;
  auto fail = [&](int rc) {
    release(e);
    return rc;
  };
  MPI_Comm_rank(comm, &e->rank);
  MPI_Comm_size(comm, &e->size);
  e->device = pick_device(comm);
  if (e->size > 1) {
    const char* m = getenv("FTAR_MPI_TRANSPORT");
    const std::string mode = m && *m ? m : "auto";
    if (mode != "rccl" && mode != "ipc" && mode != "auto") return fail(MPI_ERR_ARG);
    int rccl_ok = 0;
    if (mode != "ipc") {
      ftar_unique_id_t id;
      memset(&id, 0, sizeof id);
      int ok = e->rank == 0 ? ftar_get_unique_id(&id) == FTAR_SUCCESS : 1;
      MPI_Bcast(&ok, 1, MPI_INT, 0, comm);
      if (ok) {
        MPI_Bcast(&id, (int)sizeof id, MPI_BYTE, 0, comm);
        rccl_ok = ftar_comm_init_rank(&e->comm, e->size, id, e->rank, e->device) == FTAR_SUCCESS;
      }
      int all_ok = rccl_ok;
      MPI_Allreduce(&rccl_ok, &all_ok, 1, MPI_INT, MPI_MIN, comm);  // every rank takes the same path
      if (!all_ok && e->comm) {
        ftar_comm_destroy(e->comm);
        e->comm = nullptr;
      }
      rccl_ok = all_ok;
      if (!rccl_ok && mode == "rccl") return fail(MPI_ERR_OTHER);
    }
    if (!rccl_ok) {
      if (MPI_Comm_dup(comm, &e->boot) != MPI_SUCCESS) return fail(MPI_ERR_OTHER);
      if (ftar_comm_init_host(&e->comm, e->size, e->rank, e->device, mpi_allgather, &e->boot) != FTAR_SUCCESS)
        return fail(MPI_ERR_OTHER);
      int pd = 0;
      if (ftar_comm_get_peer_direct(e->comm, &pd) == FTAR_SUCCESS && pd == 0)
        (void)ftar_comm_set_peer_direct(e->comm, FTAR_PEER_READ);
      e->ipc = true;
    }
  }
  e->ready = true;
  return MPI_SUCCESS;
}

// get_stages runs first on every call (mpi_mod.hpp:1732), so an invalid
// FT_TOPO fails every call, a 1-rank call (whose copy never reaches the
// engine) included.  The engine re-checks, per call, for C-ABI callers.
// The last verdict per (FT_TOPO, FT_LONELY, size) is kept: a lonely layout's
// check builds every rank's plan, and an unchanged environment should cost
// two getenv per call.
int check_env_topo(int nranks) {
  const char* t = getenv("FT_TOPO");
  const char* l = getenv("FT_LONELY");
  if ((!t || !*t) && (!l || !*l || !strcmp(l, "0"))) return MPI_SUCCESS;  // unset: the cost model
  static std::mutex mu;
  static std::string last_t, last_l;
  static int last_n = -1, last_rc = MPI_SUCCESS;
  std::lock_guard<std::mutex> g(mu);
  const std::string st = t ? t : "", sl = l ? l : "";
  if (nranks != last_n || st != last_t || sl != last_l) {
    ftar_topo_t x;
    last_rc = ftar_topo_parse(t, l, nranks, &x) == FTAR_SUCCESS ? MPI_SUCCESS : MPI_ERR_ARG;
    last_n = nranks;
    last_t = st;
    last_l = sl;
  }
  return last_rc;
}

// FTAR_COST_FILE (the node's calibration, ftar.h): a file that does not parse fails the call with
// MPI_ERR_ARG on every rank before anything is brought up, rather than the auto transport taking it for an
// RCCL failure; the last verdict per path is kept
int check_cost_file() {
  const char* f = getenv("FTAR_COST_FILE");
  if (!f || !*f) return MPI_SUCCESS;
  static std::mutex mu;
  static std::string last;
  static int last_rc = MPI_SUCCESS;
  std::lock_guard<std::mutex> g(mu);
  if (last != f) {
    last = f;
    last_rc = ftar_cost_load(f) == FTAR_SUCCESS ? MPI_SUCCESS : MPI_ERR_ARG;
  }
  return last_rc;
}

// FTAR_REDUCE_CUS (a CU share for the reduce stream) is refused on RCCL communicators (ftar.h), so with a
// transport that may be RCCL (rccl, or auto) it fails the call with MPI_ERR_ARG on every rank before the
// bring-up -- else the RCCL communicator's init would fail and auto would take that for an RCCL failure and
// switch every rank to ipc.  With FTAR_MPI_TRANSPORT=ipc the knob applies.
int check_reduce_cus() {
  const char* cus = getenv("FTAR_REDUCE_CUS");
  if (!cus || !*cus || atoi(cus) == 0) return MPI_SUCCESS;
  const char* m = getenv("FTAR_MPI_TRANSPORT");
  return m && !strcmp(m, "ipc") ? MPI_SUCCESS : MPI_ERR_ARG;
}

// before the communicator's bring-up, as get_stages precedes everything in the
// reference's call: a bad FT_TOPO fails every rank alike, GPU or not (and so
// does a calibration file that does not parse, or a CU share RCCL refuses)
int check_topo_first(MPI_Comm comm) {
  int size = 1;
  if (MPI_Comm_size(comm, &size) != MPI_SUCCESS) return MPI_ERR_COMM;
  int rc = check_env_topo(size);
  if (rc == MPI_SUCCESS) rc = check_cost_file();
  if (rc == MPI_SUCCESS && size > 1) rc = check_reduce_cus();
  return rc;
}

int status_to_mpi(ftar_status_t st) {
  switch (st) {
    case FTAR_SUCCESS: return MPI_SUCCESS;
    case FTAR_ERR_NO_MEMORY: return MPI_ERR_NO_MEM;
    case FTAR_ERR_INVALID_TOPO:
    case FTAR_ERR_INVALID_ARG: return MPI_ERR_ARG;
    default: return MPI_ERR_OTHER;
  }
}

// device + stream on first GPU use (a 1-rank communicator's host path never needs them)
int ensure_stream(Entry* e) {
  if (hipSetDevice(e->device) != hipSuccess) return MPI_ERR_OTHER;
  if (!e->stream && hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) return MPI_ERR_OTHER;
  return MPI_SUCCESS;
}

// the registration covering [p, p + bytes), or end()
std::map<uintptr_t, Registration>::iterator covering(const void* p, size_t bytes) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  auto it = g_registered.upper_bound(a);
  if (it == g_registered.begin()) return g_registered.end();
  --it;
  return a + bytes <= it->first + it->second.bytes ? it : g_registered.end();
}

bool auto_register() {
  static const bool on = getenv("FTAR_MPI_REGISTER") && atoi(getenv("FTAR_MPI_REGISTER")) != 0;
  return on;
}

size_t auto_register_max() {
  static const size_t m = getenv("FTAR_MPI_REGISTER_MAX") ? strtoull(getenv("FTAR_MPI_REGISTER_MAX"), nullptr, 0) : 4;
  return m;
}

// Pin (or find pinned) the range for one call; returns the registration's key
// to release after the call, or 0 (pageable copies).
uintptr_t acquire_pinned(const void* p, size_t bytes) {
  if (!p || !bytes) return 0;
  std::lock_guard<std::mutex> g(g_mu);
  auto it = covering(p, bytes);
  if (it == g_registered.end()) {
    if (!auto_register()) return 0;
    // evict least recently used automatic registrations nobody is copying through
    size_t nauto = 0;
    for (auto& kv : g_registered) nauto += kv.second.automatic;
    while (nauto >= std::max<size_t>(1, auto_register_max())) {
      auto lru = g_registered.end();
      for (auto j = g_registered.begin(); j != g_registered.end(); ++j)
        if (j->second.automatic && !j->second.in_use &&
            (lru == g_registered.end() || j->second.last_use < lru->second.last_use))
          lru = j;
      if (lru == g_registered.end()) return 0;  // all busy: this call copies pageable
      (void)hipHostUnregister(reinterpret_cast<void*>(lru->first));
      g_registered.erase(lru);
      --nauto;
    }
    if (hipHostRegister(const_cast<void*>(p), bytes, hipHostRegisterDefault) != hipSuccess) {
      (void)hipGetLastError();  // overlaps a registration, or not registrable: pageable copies still work
      return 0;
    }
    Registration r;
    r.bytes = bytes;
    r.automatic = true;
    it = g_registered.emplace(reinterpret_cast<uintptr_t>(p), r).first;
  }
  ++it->second.in_use;
  it->second.last_use = ++g_tick;
  return it->first;
}

void release_pinned(uintptr_t key) {
  if (!key) return;
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_registered.find(key);
  if (it != g_registered.end() && it->second.in_use > 0) --it->second.in_use;
}

struct Pinned {  // the call's source and destination registrations, released on every return path
  uintptr_t a = 0, b = 0;
  ~Pinned() {
    release_pinned(a);
    release_pinned(b);
  }
};

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
  Entry* e;
  int rc = lookup(comm, &e);
  if (rc != MPI_SUCCESS) return rc;
  std::lock_guard<std::mutex> g(e->mu);
  if ((rc = init_entry(e, comm)) == MPI_SUCCESS) *out = e->comm;
  return rc;
}

int MPI_Allreduce_FT(const void* sendbuf, void* recvbuf, int count, MPI_Datatype datatype, MPI_Op op,
                     MPI_Comm comm) {
  ftar_dtype_t dt;
  ftar_op_t fo;
  if (ftar_mpi_dtype(datatype, &dt) != MPI_SUCCESS) return MPI_ERR_TYPE;
  if (ftar_mpi_op(op, &fo) != MPI_SUCCESS) return MPI_ERR_OP;
  if (count < 0 || (!recvbuf && count)) return MPI_ERR_ARG;
  Entry* e;
  int rc = lookup(comm, &e);
  if (rc != MPI_SUCCESS) return rc;
  if ((rc = check_topo_first(comm)) != MPI_SUCCESS) return rc;
  std::lock_guard<std::mutex> g(e->mu);
  if ((rc = init_entry(e, comm)) != MPI_SUCCESS) return rc;
  const size_t bytes = (size_t)count * ftar_dtype_size(dt);
  const void* src = sendbuf == MPI_IN_PLACE ? recvbuf : sendbuf;
  if (e->size <= 1) {  // mpi_mod.hpp:1739-1746
    if (src != recvbuf && bytes) memcpy(recvbuf, src, bytes);
    return MPI_SUCCESS;
  }
  if ((rc = ensure_stream(e)) != MPI_SUCCESS) return rc;
  Pinned pin;
  pin.a = acquire_pinned(src, bytes);
  if (src != recvbuf) pin.b = acquire_pinned(recvbuf, bytes);
  const ftar_status_t st = ftar_allreduce_host(src == recvbuf ? nullptr : src, recvbuf, (size_t)count, dt, fo,
                                               nullptr, e->comm, e->stream);
  if (st != FTAR_SUCCESS) return status_to_mpi(st);
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
  Entry* e;
  int rc = lookup(comm, &e);
  if (rc != MPI_SUCCESS) return rc;
  if ((rc = check_topo_first(comm)) != MPI_SUCCESS) return rc;
  std::lock_guard<std::mutex> g(e->mu);
  if ((rc = init_entry(e, comm)) != MPI_SUCCESS) return rc;
  if ((rc = ensure_stream(e)) != MPI_SUCCESS) return rc;
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : e->stream;
  const void* src = sendbuf == MPI_IN_PLACE ? nullptr : sendbuf;
  if (e->size <= 1) {
    if (src && src != recvbuf && count &&
        hipMemcpyAsync(recvbuf, src, (size_t)count * ftar_dtype_size(dt), hipMemcpyDeviceToDevice, s) != hipSuccess)
      return MPI_ERR_OTHER;
  } else {
    const ftar_status_t st = ftar_allreduce(src, recvbuf, (size_t)count, dt, fo, nullptr, e->comm, s);
    if (st != FTAR_SUCCESS) return status_to_mpi(st);
  }
  if (!stream && hipStreamSynchronize(s) != hipSuccess) return MPI_ERR_OTHER;
  return MPI_SUCCESS;
}

int MPI_Allreduce_FT_register(const void* buf, size_t bytes) {
  if (!buf || !bytes) return MPI_ERR_ARG;
  std::lock_guard<std::mutex> g(g_mu);
  const uintptr_t key = reinterpret_cast<uintptr_t>(buf);
  auto it = covering(buf, bytes);
  if (it != g_registered.end()) {  // already pinned (explicitly, or automatically: now the caller's)
    it->second.automatic = false;
    return MPI_SUCCESS;
  }
  if (hipHostRegister(const_cast<void*>(buf), bytes, hipHostRegisterDefault) != hipSuccess) {
    (void)hipGetLastError();
    return MPI_ERR_OTHER;
  }
  Registration r;
  r.bytes = bytes;
  g_registered[key] = r;
  return MPI_SUCCESS;
}

int MPI_Allreduce_FT_unregister(const void* buf) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_registered.find(reinterpret_cast<uintptr_t>(buf));
  if (it == g_registered.end()) return MPI_ERR_ARG;
  if (it->second.in_use) return MPI_ERR_PENDING;  // a call is copying through it right now
  (void)hipHostUnregister(reinterpret_cast<void*>(it->first));
  g_registered.erase(it);
  return MPI_SUCCESS;
}

int MPI_Allreduce_FT_finalize(void) {
  std::vector<Entry*> live;
  int keyval;
  {
    std::lock_guard<std::mutex> g(g_mu);
    live.assign(g_live.begin(), g_live.end());
    keyval = g_keyval;
  }
  // deleting the attribute runs delete_entry, which releases the entry
  for (Entry* e : live) MPI_Comm_delete_attr(e->owner, keyval);
  std::lock_guard<std::mutex> g(g_mu);
  if (g_keyval != MPI_KEYVAL_INVALID) MPI_Comm_free_keyval(&g_keyval);
  for (auto& kv : g_registered) (void)hipHostUnregister(reinterpret_cast<void*>(kv.first));
  g_registered.clear();
  return MPI_SUCCESS;
}

}  // extern "C"
