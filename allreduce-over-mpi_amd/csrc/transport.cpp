// Transports of the FlexTree engine: point-to-point, stream-ordered byte moves.
//
// The reference moves every block with MPI_Isend/MPI_Irecv, tag 0, matched in
// posting order per peer pair, and then blocks in MPI_Waitall + MPI_Barrier
// (mpi_mod.hpp:1254-1305, :1576-1595, :1696-1712).  Here a stage's moves are
// one group of non-blocking, stream-ordered p2p operations; completion is a
// stream event, never a host wait or a barrier.
//
//   RcclTransport   one process per GPU: ncclSend/ncclRecv inside
//                   ncclGroupStart/End over xGMI (the product path).
//   LocalTransport  N ranks inside one process (one host thread per rank):
//                   the receiver enqueues a device copy from the sender's
//                   buffer on its own stream, ordered after the sender's
//                   "ready" event; the sender's stream then waits for the
//                   receiver's "copied" event.  Same per-pair FIFO matching,
//                   same stream semantics as RCCL p2p, so the engine code
//                   above it is identical; used to run multi-rank schedules
//                   on a single GPU (tests) and in single-process groups.
#include <rccl/rccl.h>

#include <unistd.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <random>

#include "ftar_internal.h"

namespace ftar {

bool ipc_size_guard() {
  static const bool on = [] {
    if (const char* e = getenv("FTAR_IPC_SIZE_GUARD")) return *e != '0';
    int v = 0;
    return hipRuntimeGetVersion(&v) != hipSuccess || v < 70200000;  // major*1e7 + minor*1e5 + patch
  }();
  return on;
}

// Exportable sizes: at least 2 MiB, because the runtime sub-allocates small
// hipMalloc requests out of a shared block that hipMemGetAddressRange / IPC
// export do not see as an allocation of its own (a 4-byte exchange buffer for a
// one-element bucket failed "named symbol not found"); and round past sizes
// with bit 31 set where the runtime blocks opening them (ipc_size_guard).
size_t ipc_safe_size(size_t bytes) {
  const size_t bit31 = size_t(1) << 31, mask4g = (size_t(1) << 32) - 1, min_bytes = size_t(2) << 20;
  bytes = std::max(bytes, min_bytes);
  return (ipc_size_guard() && (bytes & bit31)) ? (bytes | mask4g) + 1 : bytes;  // up to the next 4 GiB
}

namespace {
std::mutex g_tokens_mu;
std::map<const void*, std::array<uint64_t, 2>> g_tokens;  // stamped buffers (owned exchange/bounce buffers)
}

void forget_token(const void* p) {
  std::lock_guard<std::mutex> g(g_tokens_mu);
  g_tokens.erase(p);
}

ftar_status_t alloc_exportable(size_t bytes, bool ipc, void** out, size_t* got) {
  const size_t want = ipc ? ipc_safe_size(bytes) : bytes;
  *out = nullptr;
  *got = 0;
  std::vector<void*> set_aside;
  ftar_status_t st = FTAR_ERR_HIP;
  for (int attempt = 0; attempt < 4; ++attempt) {
    void* fresh = nullptr;
    const hipError_t me = hipMalloc(&fresh, want);
    if (me != hipSuccess) {
      (void)hipGetLastError();
      set_error("hipMalloc of " + std::to_string(want) + " bytes failed", __FILE__, __LINE__);
      if (me == hipErrorOutOfMemory) st = FTAR_ERR_NO_MEMORY;
      break;
    }
    IpcRef probe;
    if (!ipc || ipc_export(fresh, &probe) == FTAR_SUCCESS) {
      *out = fresh;
      *got = want;
      st = FTAR_SUCCESS;
      break;
    }
    trace("%p not exportable, allocating another", fresh);
    set_aside.push_back(fresh);
  }
  for (void* p : set_aside) hip_ignore(hipFree(p));
  return st;
}

ftar_status_t ipc_export(const void* p, IpcRef* out) {
  memset(out, 0, sizeof *out);
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  FTAR_CHECK_HIP(hipMemGetAddressRange(&base, &size, const_cast<void*>(p)));
  trace("ipc_export %p: allocation %p + %zu bytes", p, (void*)base, size);
  if (ipc_size_guard() && (size & (size_t(1) << 31))) {
    set_error("IPC export of a " + std::to_string(size) +
                  "-byte allocation refused: this HIP runtime blocks in hipIpcOpenMemHandle for sizes with bit 31 "
                  "set (FTAR_IPC_SIZE_GUARD)",
              __FILE__, __LINE__);
    return FTAR_ERR_UNSUPPORTED;
  }
  out->offset = static_cast<uint64_t>(static_cast<const char*>(p) - static_cast<const char*>(base));
  const hipError_t e = hipIpcGetMemHandle(&out->handle, base);
  if (e != hipSuccess) {
    (void)hipGetLastError();  // not sticky: the next launch check must not see it
    memset(&out->handle, 0, sizeof out->handle);
    set_error(std::string("hipIpcGetMemHandle: ") + hipGetErrorString(e), __FILE__, __LINE__);
    trace("ipc_export %p failed: %s", p, hipGetErrorString(e));
    return FTAR_ERR_HIP;
  }
  out->size = size;
  {
    std::lock_guard<std::mutex> g(g_tokens_mu);
    auto it = g_tokens.find(p);
    if (it != g_tokens.end()) {
      out->stamped = 1;
      out->token[0] = it->second[0];
      out->token[1] = it->second[1];
    }
  }
  if (!out->stamped && size - out->offset >= sizeof out->token) {
    // a caller's buffer (registration): its first 16 bytes as they are now -- the importers must read the
    // same through their mappings (the buffer may not be written while it is being registered)
    if (hipMemcpy(out->token, p, sizeof out->token, hipMemcpyDeviceToHost) == hipSuccess) out->stamped = 2;
    else (void)hipGetLastError();
  }
  out->valid = 1;
  return FTAR_SUCCESS;
}

ftar_status_t stamp_token(void* p) {
  std::array<uint64_t, 2> t;
  {
    std::lock_guard<std::mutex> g(g_tokens_mu);
    static std::mt19937_64 rng(std::random_device{}() ^ (uint64_t)getpid() << 32);
    t = {rng(), rng()};
  }
  FTAR_CHECK_HIP(hipMemcpy(p, t.data(), sizeof t, hipMemcpyHostToDevice));
  std::lock_guard<std::mutex> g(g_tokens_mu);
  g_tokens[p] = t;
  return FTAR_SUCCESS;
}

ftar_status_t ipc_import(const IpcRef& ref, void** base, char** p) {
  if (ref.valid != 1) {
    set_error("ipc_import: the peer's export failed", __FILE__, __LINE__);
    return FTAR_ERR_HIP;
  }
  trace("ipc_import: open (offset %llu)", (unsigned long long)ref.offset);
  FTAR_CHECK_HIP(hipIpcOpenMemHandle(base, ref.handle, hipIpcMemLazyEnablePeerAccess));
  *p = static_cast<char*>(*base) + ref.offset;
  // verify the mapping: the runtime has been seen to map the wrong memory after regrowth
  std::string bad;
  hipDeviceptr_t b2 = nullptr;
  size_t sz = 0;
  if (hipMemGetAddressRange(&b2, &sz, *p) == hipSuccess) {
    if (sz < ref.size) bad = "size " + std::to_string(sz) + " < " + std::to_string(ref.size);  // (rounding up is fine)
  } else {
    (void)hipGetLastError();
  }
  if (bad.empty() && ref.stamped) {
    uint64_t got[2] = {0, 0};
    if (hipMemcpy(got, *p, sizeof got, hipMemcpyDeviceToHost) != hipSuccess) {
      (void)hipGetLastError();  // cannot read it back here: keep the mapping unverified rather than lose it
      trace("ipc_import: mapping at %p not verifiable (token unreadable)", *base);
    } else if (got[0] != ref.token[0] || got[1] != ref.token[1]) {
      bad = "token mismatch";
    }
  }
  if (!bad.empty()) {
    trace("ipc_import: mapping at %p rejected (%s)", *base, bad.c_str());
    hip_ignore(hipIpcCloseMemHandle(*base));
    *base = nullptr;
    *p = nullptr;
    set_error("ipc_import: the mapping does not show the peer's buffer (" + bad + ")", __FILE__, __LINE__);
    return FTAR_ERR_HIP;
  }
  trace("ipc_import: mapped at %p (verified)", *base);
  return FTAR_SUCCESS;
}

// ---------------------------------------------------------------------------
// RCCL
// ---------------------------------------------------------------------------
namespace {

// ncclGetLastError(NULL) adds RCCL's own detail of the failure (which peer, which transport) to the
// status string: one driver record of a failed first RCCL contact then says why (bench.py gathers every
// rank's ftar_last_error)
#define FTAR_CHECK_NCCL(expr)                                                                       \
  do {                                                                                              \
    ncclResult_t _r = (expr);                                                                       \
    if (_r != ncclSuccess) {                                                                        \
      const char* _d = ncclGetLastError(nullptr);                                                   \
      ::ftar::set_error(std::string(#expr) + ": " + ncclGetErrorString(_r) +                        \
                            (_d && *_d ? std::string(" (") + _d + ")" : std::string()),             \
                        __FILE__, __LINE__);                                                        \
      return FTAR_ERR_RCCL;                                                                         \
    }                                                                                               \
  } while (0)

// Peer allocations imported into this process: one IPC mapping per allocation
// (two registered buffers may share one), reference-counted by the pointers
// handed out, so closing one pointer never unmaps memory another still uses.
// Shared by the RCCL and the host-bootstrapped transports.
class PeerImports {
 public:
  ftar_status_t open(const IpcRef& ref, char** out) {
    const std::string key(reinterpret_cast<const char*>(&ref.handle), sizeof ref.handle);
    auto it = imports_.find(key);
    if (it == imports_.end()) {
      void* base = nullptr;
      char* p = nullptr;
      FTAR_RETURN_IF(ipc_import(ref, &base, &p));
      it = imports_.emplace(key, Import{base, 0}).first;
    }
    ++it->second.refs;
    *out = static_cast<char*>(it->second.base) + ref.offset;
    handed_.emplace(*out, key);
    return FTAR_SUCCESS;
  }
  void close(char* p) {
    auto h = handed_.find(p);
    if (h == handed_.end()) return;
    auto it = imports_.find(h->second);
    handed_.erase(h);
    if (it != imports_.end() && --it->second.refs == 0) {
      trace("ipc close %p", it->second.base);
      hip_ignore(hipIpcCloseMemHandle(it->second.base));
      imports_.erase(it);
    }
  }
  // every peer pointer of a map_peers result (the own slot is not an import)
  void close_all(std::vector<char*>* peers, int rank) {
    for (int q = 0; q < (int)peers->size(); ++q)
      if (q != rank && (*peers)[q]) close((*peers)[q]);
    peers->clear();
  }

 private:
  struct Import {
    void* base;
    int refs;
  };
  std::map<std::string, Import> imports_;     // peer allocation (IPC handle bytes) -> its mapping here
  std::multimap<char*, std::string> handed_;  // peer pointer handed out -> its allocation
};

class RcclTransport final : public Transport {
 public:
  explicit RcclTransport(ncclComm_t c) : comm_(c) {
    if (ncclCommCount(comm_, &nranks_) != ncclSuccess || nranks_ < 1) nranks_ = 1;
    // the agreement's buffer and stream exist before any agreement is attempted, so a rank never leaves
    // its peers waiting in that collective because an allocation failed at its start
    if (hipMalloc(&agree_buf_, kAgreeBytes * (size_t)(nranks_ + 1) + 2 * (size_t)nranks_) != hipSuccess ||
        hipStreamCreateWithFlags(&agree_s_, hipStreamNonBlocking) != hipSuccess) {
      (void)hipGetLastError();
      agree_ready_ = false;
    }
  }
  ~RcclTransport() override {
    if (comm_ && !aborted_.load()) ncclCommDestroy(comm_);
    if (agree_s_) hip_ignore(hipStreamDestroy(agree_s_));
    if (agree_buf_) hip_ignore(hipFree(agree_buf_));
    if (scratch_) hip_ignore(hipFree(scratch_));
  }
  bool first_contact_blocks() const override { return true; }
  // one byte each way with every peer in one group, waited for: RCCL connects a p2p pair lazily, inside the
  // ncclGroupEnd of its first ncclSend/ncclRecv, and that connection handshake blocks the host until the peer
  // makes the same call (tools/rccl_order: two communicators whose first exchanges were issued in opposite
  // orders hung there); done once at a communicator's first contact, no later call blocks on it
  ftar_status_t connect_peers(int rank) override {
    if (nranks_ < 2) return FTAR_SUCCESS;
    if (!agree_ready_) {
      set_error("RCCL transport: no agreement buffer (allocation at bring-up failed)", __FILE__, __LINE__);
      return FTAR_ERR_NO_MEMORY;
    }
    char* base = static_cast<char*>(agree_buf_) + kAgreeBytes * (size_t)(nranks_ + 1);
    bool ok = ncclGroupStart() == ncclSuccess;
    for (int q = 0; q < nranks_ && ok; ++q)
      if (q != rank)
        ok = ncclSend(base + q, 1, ncclUint8, q, comm_, agree_s_) == ncclSuccess &&
             ncclRecv(base + nranks_ + q, 1, ncclUint8, q, comm_, agree_s_) == ncclSuccess;
    ok = ncclGroupEnd() == ncclSuccess && ok;
    ok = ok && hipStreamSynchronize(agree_s_) == hipSuccess;
    if (!ok) {
      set_error("RCCL transport: connecting the peers (one byte each way) failed", __FILE__, __LINE__);
      return FTAR_ERR_RCCL;
    }
    return FTAR_SUCCESS;
  }
  // comm_ itself is never cleared: the first-contact helper thread may still be reading it inside an RCCL
  // call, which the abort makes return; the destructor, which runs after that helper has
  // finished, then skips ncclCommDestroy
  void abort() override {
    if (comm_ && !aborted_.exchange(true)) ncclCommAbort(comm_);
  }
  // a 4-byte all-reduce: complete on any rank's stream only once every rank's
  // stream has reached it
  ftar_status_t barrier(hipStream_t s) override {
    FTAR_RETURN_IF(ensure_scratch());
    FTAR_CHECK_NCCL(ncclAllReduce(scratch_, scratch_, 1, ncclInt32, ncclSum, comm_, s));
    return FTAR_SUCCESS;
  }
  // IPC references (allocation handle + offset) of every rank's pointer,
  // all-gathered over RCCL, opened here (dmabuf IPC; peer access enabled
  // lazily by the runtime)
  ftar_status_t map_peers(void* mine, int rank, int nranks, std::vector<char*>* peers) override {
    if (nranks != nranks_ || rank < 0 || rank >= nranks) return FTAR_ERR_INVALID_ARG;
    FTAR_RETURN_IF(ensure_scratch());
    IpcRef ref;
    std::string why;
    if (ipc_export(mine, &ref) != FTAR_SUCCESS) why = std::string("rank ") + std::to_string(rank) + ": " + last_error();
    std::vector<IpcRef> all(nranks);
    char* dev = static_cast<char*>(scratch_) + 256;  // nranks refs after the barrier and agreement words
    hipStream_t s;
    FTAR_CHECK_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    ftar_status_t st = FTAR_SUCCESS;
    if (hipMemcpyAsync(dev + (size_t)rank * sizeof ref, &ref, sizeof ref, hipMemcpyHostToDevice, s) != hipSuccess ||
        ncclAllGather(dev + (size_t)rank * sizeof ref, dev, sizeof ref, ncclUint8, comm_, s) != ncclSuccess ||
        hipMemcpyAsync(all.data(), dev, (size_t)nranks * sizeof ref, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
      set_error("peer map: handle exchange failed", __FILE__, __LINE__);
      st = FTAR_ERR_RCCL;
    }
    hip_ignore(hipStreamDestroy(s));
    FTAR_RETURN_IF(st);
    peers->assign(nranks, nullptr);
    for (int q = 0; q < nranks && why.empty(); ++q)  // a failed export anywhere: nobody opens anything
      if (all[q].valid != 1) why = std::string("rank ") + std::to_string(q) + " could not export its buffer";
    // The ranks open the peers' handles one rank at a time (a precaution
    // taken while chasing the 2 GiB open hang, ipc_size_guard, which turned
    // out to be a runtime size bug; turns cost P host agreements per mapping,
    // nothing per call).  Each turn ends with a host-side
    // agreement on the failures so far, so every rank also learns whether
    // every rank mapped every peer (a rank that failed alone would otherwise
    // leave the others waiting in the next barrier).
    int failed = 0;
    for (int turn = 0; turn < nranks; ++turn) {
      if (turn == rank && why.empty()) {
        for (int q = 0; q < nranks; ++q) {
          if (q == rank) {
            (*peers)[q] = static_cast<char*>(mine);
            continue;
          }
          if (imports_.open(all[q], &(*peers)[q]) != FTAR_SUCCESS) {
            why = std::string("rank ") + std::to_string(q) + ": " + last_error();
            break;
          }
        }
      }
      FTAR_RETURN_IF(agree_failures(why.empty() ? 0 : 1, &failed));
    }
    if (failed) {
      unmap_peers(peers, rank);
      set_error(why.empty() ? std::to_string(failed) + " peer rank(s) could not map the exchange buffers" : why,
                __FILE__, __LINE__);
      return FTAR_ERR_HIP;
    }
    return FTAR_SUCCESS;
  }
  void unmap_peers(std::vector<char*>* peers, int rank) override { imports_.close_all(peers, rank); }
  ftar_status_t group_start() override {
    FTAR_CHECK_NCCL(ncclGroupStart());
    return FTAR_SUCCESS;
  }
  ftar_status_t send(const void* buf, size_t bytes, int peer, hipStream_t s) override {
    FTAR_CHECK_NCCL(ncclSend(buf, bytes, ncclUint8, peer, comm_, s));
    return FTAR_SUCCESS;
  }
  ftar_status_t recv(void* buf, size_t bytes, int peer, hipStream_t s) override {
    FTAR_CHECK_NCCL(ncclRecv(buf, bytes, ncclUint8, peer, comm_, s));
    return FTAR_SUCCESS;
  }
  ftar_status_t group_end() override {
    FTAR_CHECK_NCCL(ncclGroupEnd());
    return FTAR_SUCCESS;
  }
  const char* name() const override { return "rccl"; }
  bool uses_ipc() const override { return true; }
  bool masked_reduce_stream_ok() const override { return false; }
  ftar_status_t allgather(const void* send, void* recv, size_t bytes, int rank, int nranks, hipStream_t s) override {
    (void)rank;
    (void)nranks;
    FTAR_CHECK_NCCL(ncclAllGather(send, recv, bytes, ncclUint8, comm_, s));
    return FTAR_SUCCESS;
  }
  ftar_status_t native_allreduce(const void* send, void* recv, size_t count, ftar_dtype_t dt, ftar_op_t op,
                                 hipStream_t s) override {
    ncclDataType_t t;
    switch (dt) {
      case FTAR_UINT8: t = ncclUint8; break;
      case FTAR_INT8: t = ncclInt8; break;
      case FTAR_INT32: t = ncclInt32; break;
      case FTAR_INT64: t = ncclInt64; break;
      case FTAR_FLOAT32: t = ncclFloat32; break;
      case FTAR_FLOAT64: t = ncclFloat64; break;
      case FTAR_BFLOAT16: t = ncclBfloat16; break;
      default: return FTAR_ERR_UNSUPPORTED;
    }
    if (op != FTAR_SUM) return FTAR_ERR_UNSUPPORTED;
    FTAR_CHECK_NCCL(ncclAllReduce(send ? send : recv, recv, count, t, ncclSum, comm_, s));
    return FTAR_SUCCESS;
  }

  void* rccl_register(void* buf, size_t bytes) override {
    void* h = nullptr;
    if (ncclCommRegister(comm_, buf, bytes, &h) != ncclSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    return h;
  }
  void rccl_deregister(void* handle) override {
    if (handle && !aborted_.load()) (void)ncclCommDeregister(comm_, handle);
  }
  // every rank's bytes through one ncclAllGather on a private stream (host-blocking; communicator
  // bring-up only)
  ftar_status_t agree(const void* mine, size_t bytes, bool* same) override {
    if (bytes > kAgreeBytes || !agree_ready_) {
      set_error("settings agreement: no agreement buffer, or more than 256 bytes to agree on", __FILE__, __LINE__);
      return FTAR_ERR_INTERNAL;
    }
    char* dev = static_cast<char*>(agree_buf_);
    std::vector<char> all((size_t)nranks_ * bytes);
    const bool ok = hipMemcpyAsync(dev, mine, bytes, hipMemcpyHostToDevice, agree_s_) == hipSuccess &&
                    ncclAllGather(dev, dev + kAgreeBytes, bytes, ncclUint8, comm_, agree_s_) == ncclSuccess &&
                    hipMemcpyAsync(all.data(), dev + kAgreeBytes, all.size(), hipMemcpyDeviceToHost, agree_s_) ==
                        hipSuccess &&
                    hipStreamSynchronize(agree_s_) == hipSuccess;
    if (!ok) {
      set_error("settings agreement: the all-gather failed", __FILE__, __LINE__);
      return FTAR_ERR_RCCL;
    }
    *same = true;
    for (int q = 0; q < nranks_; ++q) *same = *same && !memcmp(all.data() + (size_t)q * bytes, mine, bytes);
    return FTAR_SUCCESS;
  }

 private:
  static constexpr size_t kAgreeBytes = 256;
  void* agree_buf_ = nullptr;  // one agreement per rank (all-gathered) + the connection bytes
  hipStream_t agree_s_ = nullptr;
  bool agree_ready_ = true;

  // sum of every rank's `mine` (host-blocking, on a private stream)
  ftar_status_t agree_failures(int mine, int* total) {
    int* word = reinterpret_cast<int*>(static_cast<char*>(scratch_) + 128);
    hipStream_t s;
    FTAR_CHECK_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    bool ok = hipMemcpyAsync(word, &mine, sizeof mine, hipMemcpyHostToDevice, s) == hipSuccess &&
              ncclAllReduce(word, word, 1, ncclInt32, ncclSum, comm_, s) == ncclSuccess &&
              hipMemcpyAsync(total, word, sizeof *total, hipMemcpyDeviceToHost, s) == hipSuccess &&
              hipStreamSynchronize(s) == hipSuccess;
    hip_ignore(hipStreamDestroy(s));
    if (!ok) {
      set_error("peer map: failure agreement failed", __FILE__, __LINE__);
      return FTAR_ERR_RCCL;
    }
    return FTAR_SUCCESS;
  }
  // barrier word, agreement word, one IPC reference per rank (map_peers all-gathers nranks of them)
  ftar_status_t ensure_scratch() {
    if (!scratch_) FTAR_CHECK_HIP(hipMalloc(&scratch_, 256 + (size_t)std::max(nranks_, 1) * sizeof(IpcRef)));
    return FTAR_SUCCESS;
  }
  ncclComm_t comm_;
  std::atomic<bool> aborted_{false};
  int nranks_ = 1;
  void* scratch_ = nullptr;
  PeerImports imports_;
};

}  // namespace

std::unique_ptr<Transport> make_rccl_transport(int nranks, const ftar_unique_id_t& id, int rank, ftar_status_t* st) {
  static_assert(sizeof(ftar_unique_id_t) == sizeof(ncclUniqueId), "unique id size");
  ncclUniqueId uid;
  memcpy(&uid, &id, sizeof(uid));
  ncclComm_t c = nullptr;
  ncclResult_t r = ncclCommInitRank(&c, nranks, uid, rank);
  if (r != ncclSuccess) {
    const char* d = ncclGetLastError(nullptr);
    set_error(std::string("ncclCommInitRank: ") + ncclGetErrorString(r) +
                  (d && *d ? std::string(" (") + d + ")" : std::string()),
              __FILE__, __LINE__);
    *st = FTAR_ERR_RCCL;
    return nullptr;
  }
  *st = FTAR_SUCCESS;
  return std::unique_ptr<Transport>(new RcclTransport(c));
}

// ---------------------------------------------------------------------------
// in-process ranks
// ---------------------------------------------------------------------------
namespace {
thread_local bool t_issue_held = false;  // this thread holds its group's issue lock (capture)
}

struct LocalHub {
  // Per-message and barrier events are recycled through a pool, never
  // destroyed before the hub: a stream capture may still refer to an event
  // after both sides dropped the message.
  // A pooled event shared by the messages of one flush: the sends of a flush on one stream share their
  // data-ready event, the receives of a flush on one stream their copies-done event (one record each
  // instead of one per message); the last holder gives it back to the pool.
  using Ev = std::shared_ptr<hipEvent_t>;
  struct Posted {
    const void* buf;
    size_t bytes;
    Ev ready;     // sender-side data ready
    Ev done;      // receiver-side copy finished (set by the receiver)
    bool taken = false;
    int device = -1;  // the sender's device
    int sender = -1;
  };
  ftar_status_t take_shared(Ev* out) {
    Ev e(new hipEvent_t(nullptr), [this](hipEvent_t* p) {
      if (*p) give_event(*p);
      delete p;
    });
    FTAR_RETURN_IF(take_event(e.get()));
    *out = std::move(e);
    return FTAR_SUCCESS;
  }
  // During a capture (this thread holds the issue lock) every record gets a
  // fresh event and used ones retire until the next uncaptured use: an event
  // re-recorded inside one capture -- on another rank's stream after a peer
  // waited on it -- made hipStreamEndCapture recurse without end
  // (tools/capture/, profiles/r02/capture/).
  ftar_status_t take_event(hipEvent_t* e) {
    {
      std::lock_guard<std::mutex> g(pool_mu);
      if (!t_issue_held && !retired.empty()) {
        pool.insert(pool.end(), retired.begin(), retired.end());
        retired.clear();
      }
      if (!t_issue_held && !pool.empty()) {
        *e = pool.back();
        pool.pop_back();
        return FTAR_SUCCESS;
      }
    }
    FTAR_CHECK_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
    return FTAR_SUCCESS;
  }
  void give_event(hipEvent_t e) {
    std::lock_guard<std::mutex> g(pool_mu);
    (t_issue_held ? retired : pool).push_back(e);
  }
  ~LocalHub() {
    // the last rendezvous rounds and any undelivered messages still hold pooled events whose deleters give
    // them back here: release them while the pool is alive, then destroy the pool (a barrier's round left
    // in `done` was given back into the destroyed pool after it, a double free on destroying a group whose
    // last call was a peer form)
    done.reset();
    pending.reset();
    wire.clear();
    for (hipEvent_t e : pool) hip_ignore(hipEventDestroy(e));
    for (hipEvent_t e : retired) hip_ignore(hipEventDestroy(e));
    pool.clear();
    retired.clear();
  }
  // Rank `rank` waits on its own condition variable (a message for it, its message taken, a rendezvous
  // complete), so a notification wakes the one thread it concerns rather than every rank's.  The wait lets
  // the other ranks' threads issue meanwhile when this one holds the issue lock (lock order: issue before mu).
  template <class Pred>
  bool wait(std::unique_lock<std::mutex>& g, int rank, Pred pred) {
    std::condition_variable& cv = rcv[rank];
    if (!t_issue_held) return cv.wait_for(g, std::chrono::seconds(120), pred);
    if (pred()) return true;
    g.unlock();
    issue.unlock();
    g.lock();
    const bool ok = cv.wait_for(g, std::chrono::seconds(120), pred);
    g.unlock();
    issue.lock();
    g.lock();
    return ok;
  }
  // every rank's value of one rendezvous (barriers, peer pointers)
  struct Round {
    std::vector<const void*> ptr;
    std::vector<std::shared_ptr<hipEvent_t>> ev;
  };
  void notify(int rank) { rcv[rank].notify_all(); }
  // After any transport failure the group is unusable: messages of the failed call may still
  // sit in `wire` and a failed sender's buffer may still be read by copies enqueued for it, so a later call
  // could pair a receive with a stale message.  fail() records the first failure and wakes every waiter;
  // every later operation of every rank is refused (destroy the group and create a new one).
  void fail(const std::string& why) {
    {
      std::lock_guard<std::mutex> g(mu);
      if (broken.empty()) broken = why.empty() ? std::string("a transport failure") : why;
    }
    for (int q = 0; q < nranks; ++q) rcv[q].notify_all();
  }
  ftar_status_t usable() {
    std::string why;
    {
      std::lock_guard<std::mutex> g(mu);
      why = broken;
    }
    if (why.empty()) return FTAR_SUCCESS;
    set_error("local transport: this group failed in an earlier call (" + why +
                  "); destroy it and create a new one",
              __FILE__, __LINE__);
    return FTAR_ERR_INTERNAL;
  }
  // whether kernels on device `dev` may read device `peer`'s memory (ftar_comm_init_local enables peer
  // access between every pair that supports it), cached per pair
  bool can_reach(int dev, int peer) {
    std::lock_guard<std::mutex> g(pool_mu);
    auto it = reach.find({dev, peer});
    if (it != reach.end()) return it->second;
    int can = 0;
    const bool ok = hipDeviceCanAccessPeer(&can, dev, peer) == hipSuccess && can;
    reach[{dev, peer}] = ok;
    return ok;
  }
  explicit LocalHub(int n) : nranks(n), rcv(new std::condition_variable[n]), pending(std::make_shared<Round>()) {
    pending->ptr.resize(n);
    pending->ev.resize(n);
  }
  // Host-side all-gather of one (pointer, event) per rank.  A generation
  // completes only when every rank arrived, so the finished Round cannot be
  // replaced before each of its ranks has taken it.
  ftar_status_t rendezvous(int rank, const void* p, std::shared_ptr<hipEvent_t> e, std::shared_ptr<Round>* out) {
    std::unique_lock<std::mutex> g(mu);
    const long my_gen = gen;
    pending->ptr[rank] = p;
    pending->ev[rank] = std::move(e);
    if (++arrived == nranks) {
      done = pending;
      pending = std::make_shared<Round>();
      pending->ptr.resize(nranks);
      pending->ev.resize(nranks);
      arrived = 0;
      ++gen;
      for (int q = 0; q < nranks; ++q) rcv[q].notify_all();
    } else if (!wait(g, rank, [&] { return gen != my_gen || !broken.empty(); })) {
      set_error("local transport: rendezvous timed out", __FILE__, __LINE__);
      return FTAR_ERR_TIMEOUT;
    } else if (gen == my_gen) {
      set_error("local transport: another rank failed during a rendezvous (" + broken + ")", __FILE__, __LINE__);
      return FTAR_ERR_INTERNAL;
    }
    *out = done;
    return FTAR_SUCCESS;
  }
  int nranks;
  std::mutex mu;
  std::unique_ptr<std::condition_variable[]> rcv;  // one per rank
  std::map<std::pair<int, int>, std::deque<std::shared_ptr<Posted>>> wire;  // (from, to)
  std::shared_ptr<Round> pending, done;
  int arrived = 0;
  long gen = 0;
  std::string broken;  // the first failure (under mu); non-empty: every later operation is refused
  std::mutex issue;  // capture of the group: one issuing thread at a time
  std::mutex pool_mu;
  std::vector<hipEvent_t> pool, retired;
  std::map<std::pair<int, int>, bool> reach;  // can_reach, under pool_mu
};

std::shared_ptr<LocalHub> make_local_hub(int nranks) { return std::make_shared<LocalHub>(nranks); }

namespace {

class LocalTransport final : public Transport {
  struct Op {
    bool is_send;
    void* buf;
    size_t bytes;
    int peer;
    hipStream_t s;
  };

 public:
  LocalTransport(std::shared_ptr<LocalHub> h, int rank) : hub_(std::move(h)), rank_(rank) {}
  ftar_status_t group_start() override {
    ++depth_;
    return FTAR_SUCCESS;
  }
  ftar_status_t send(const void* buf, size_t bytes, int peer, hipStream_t s) override {
    ops_.push_back({true, const_cast<void*>(buf), bytes, peer, s});
    return depth_ ? FTAR_SUCCESS : flush();
  }
  ftar_status_t recv(void* buf, size_t bytes, int peer, hipStream_t s) override {
    ops_.push_back({false, buf, bytes, peer, s});
    return depth_ ? FTAR_SUCCESS : flush();
  }
  ftar_status_t group_end() override {
    if (depth_ <= 0) return FTAR_ERR_INVALID_ARG;
    if (--depth_ == 0) return flush();
    return FTAR_SUCCESS;
  }
  const char* name() const override { return "local"; }
  bool capture_serially() const override { return true; }
  void capture_enter() override {
    hub_->issue.lock();
    t_issue_held = true;
  }
  void capture_leave() override {
    t_issue_held = false;
    hub_->issue.unlock();
  }
  ftar_status_t before_join() override {
    if (!t_issue_held) return FTAR_SUCCESS;
    return guarded([&] {
      std::shared_ptr<LocalHub::Round> r;
      return hub_->rendezvous(rank_, nullptr, nullptr, &r);
    });
  }
  ftar_status_t barrier(hipStream_t s) override {
    return guarded([&] { return barrier_impl(s); });
  }
  ftar_status_t map_peers(void* mine, int rank, int nranks, std::vector<char*>* peers) override {
    return guarded([&] { return map_peers_impl(mine, rank, nranks, peers); });
  }

 private:
  // refused once the group failed; a failure here breaks the group for every rank
  template <class F>
  ftar_status_t guarded(F&& fn) {
    FTAR_RETURN_IF(hub_->usable());
    const ftar_status_t st = fn();
    if (st != FTAR_SUCCESS) hub_->fail(last_error());
    return st;
  }
  // each rank's stream waits for every other rank's event recorded at the barrier
  ftar_status_t barrier_impl(hipStream_t s) {
    LocalHub* hub = hub_.get();
    auto e = std::shared_ptr<hipEvent_t>(new hipEvent_t(nullptr), [hub](hipEvent_t* p) {
      if (*p) hub->give_event(*p);
      delete p;
    });
    FTAR_RETURN_IF(hub_->take_event(e.get()));
    FTAR_CHECK_HIP(hipEventRecord(*e, s));
    std::shared_ptr<LocalHub::Round> r;
    FTAR_RETURN_IF(hub_->rendezvous(rank_, nullptr, e, &r));
    for (int q = 0; q < hub_->nranks; ++q)
      if (q != rank_) FTAR_CHECK_HIP(hipStreamWaitEvent(s, *r->ev[q], 0));
    return FTAR_SUCCESS;
  }
  // one address space: the peers' allocations are usable as they are
  ftar_status_t map_peers_impl(void* mine, int rank, int nranks, std::vector<char*>* peers) {
    (void)rank;
    std::shared_ptr<LocalHub::Round> r;
    FTAR_RETURN_IF(hub_->rendezvous(rank_, mine, nullptr, &r));
    peers->assign(nranks, nullptr);
    for (int q = 0; q < nranks; ++q) (*peers)[q] = static_cast<char*>(const_cast<void*>(r->ptr[q]));
    return FTAR_SUCCESS;
  }

  ftar_status_t flush() {
    std::vector<Op> ops;
    ops.swap(ops_);
    return guarded([&] { return flush_ops(ops); });
  }

  ftar_status_t flush_ops(std::vector<Op>& ops) {
    using Ev = LocalHub::Ev;
    // the event of a stream within this flush (sends: data ready; receives: copies done), recorded once
    auto per_stream = [](std::vector<std::pair<hipStream_t, Ev>>& v, hipStream_t st) -> Ev* {
      for (auto& x : v)
        if (x.first == st) return &x.second;
      v.emplace_back(st, nullptr);
      return &v.back().second;
    };
    // 1. publish every send, with an event marking its data ready on the sender's stream (one per stream)
    std::vector<std::pair<hipStream_t, Ev>> ready;
    std::vector<std::shared_ptr<LocalHub::Posted>> mine;
    int dev = -1;
    FTAR_CHECK_HIP(hipGetDevice(&dev));
    for (auto& o : ops) {
      if (!o.is_send) continue;
      if (o.peer == rank_ || o.peer < 0 || o.peer >= hub_->nranks) return FTAR_ERR_INVALID_ARG;
      Ev* e = per_stream(ready, o.s);
      if (!*e) {
        FTAR_RETURN_IF(hub_->take_shared(e));
        FTAR_CHECK_HIP(hipEventRecord(**e, o.s));
      }
      auto p = std::make_shared<LocalHub::Posted>();
      p->buf = o.buf;
      p->bytes = o.bytes;
      p->ready = *e;
      p->device = dev;
      p->sender = rank_;
      mine.push_back(p);
      {
        std::lock_guard<std::mutex> g(hub_->mu);
        hub_->wire[{rank_, o.peer}].push_back(p);
      }
      hub_->notify(o.peer);
    }
    // 2. issue every receive in posting order (per-pair FIFO, like MPI/RCCL): wait for the sender's data,
    // copy; then one copies-done event per receiving stream, handed to every sender of this flush
    std::vector<std::pair<hipStream_t, Ev>> done;
    std::vector<std::pair<std::shared_ptr<LocalHub::Posted>, hipStream_t>> got;
    std::vector<std::pair<hipStream_t, hipEvent_t>> waited;  // (stream, event) already waited on
    std::vector<std::pair<hipStream_t, std::vector<Segment>>> gathers;  // batched receives per stream
    auto per_stream_segs = [&](std::vector<std::pair<hipStream_t, std::vector<Segment>>>& v,
                               hipStream_t st) -> std::vector<Segment>* {
      for (auto& x : v)
        if (x.first == st) return &x.second;
      v.emplace_back(st, std::vector<Segment>());
      return &v.back().second;
    };
    // hand every message taken so far back to its sender: with its stream's copies-done event, or none if
    // this rank failed (the sender then fails too, at once, instead of waiting out the timeout)
    auto publish = [&](ftar_status_t st) -> ftar_status_t {
      if (st != FTAR_SUCCESS) {
        // a failed flush hands the senders their messages back only once the copies it already enqueued from
        // them have finished, so a failed sender that returns at once may free or reuse its buffer;
        // the receiving streams wait only on the senders' data-ready events, recorded before the senders wait
        // for anything of this flush, so these synchronisations end
        std::vector<hipStream_t> seen;
        for (auto& x : got)
          if (std::find(seen.begin(), seen.end(), x.second) == seen.end()) {
            seen.push_back(x.second);
            hip_ignore(hipStreamSynchronize(x.second));
          }
      }
      for (auto& x : got) {
        Ev* e = per_stream(done, x.second);
        if (st != FTAR_SUCCESS || *e) continue;
        st = hub_->take_shared(e);
        if (st == FTAR_SUCCESS && hipEventRecord(**e, x.second) != hipSuccess) {
          set_error("local transport: hipEventRecord failed", __FILE__, __LINE__);
          st = FTAR_ERR_HIP;
        }
      }
      {
        std::lock_guard<std::mutex> g(hub_->mu);
        for (auto& x : got) {
          if (st == FTAR_SUCCESS) x.first->done = *per_stream(done, x.second);
          x.first->taken = true;
        }
      }
      for (auto& x : got) hub_->notify(x.first->sender);
      return st;
    };
    for (auto& o : ops) {
      if (o.is_send) continue;
      std::shared_ptr<LocalHub::Posted> p;
      {
        std::unique_lock<std::mutex> g(hub_->mu);
        auto& q = hub_->wire[{o.peer, rank_}];
        if (!hub_->wait(g, rank_, [&] { return !q.empty() || !hub_->broken.empty(); })) {
          g.unlock();
          set_error("local transport: no matching send from rank " + std::to_string(o.peer), __FILE__, __LINE__);
          return publish(FTAR_ERR_TIMEOUT);
        }
        if (q.empty()) {
          const std::string why = hub_->broken;
          g.unlock();
          set_error("local transport: another rank failed (" + why + ")", __FILE__, __LINE__);
          return publish(FTAR_ERR_INTERNAL);
        }
        p = q.front();
        q.pop_front();
      }
      got.emplace_back(p, o.s);
      if (p->bytes != o.bytes) {
        set_error("local transport: message size mismatch", __FILE__, __LINE__);
        return publish(FTAR_ERR_INTERNAL);
      }
      const std::pair<hipStream_t, hipEvent_t> w{o.s, *p->ready};
      if (std::find(waited.begin(), waited.end(), w) == waited.end()) {
        if (hipStreamWaitEvent(o.s, *p->ready, 0) != hipSuccess) {
          set_error("local transport: hipStreamWaitEvent failed", __FILE__, __LINE__);
          return publish(FTAR_ERR_HIP);
        }
        waited.push_back(w);
      }
      // A receive from a rank on this device is ftar's own copy kernel, one launch per receive (launch_copy:
      // the LDS-staged copy when co-aligned): 5-6 % faster than the runtime's blit at the C4 bucket with 8
      // ranks on one GPU (profiles/r05/engine_local/ab2_*, 3 interleaved rounds); one launch per piece group
      // instead lost 2 % (it filled the GPU, and the folds stopped overlapping the copies).  The receives
      // from other devices this device can reach go into one multi-segment copy per stream, launched once
      // every one of them is waited for: its workgroups interleave the segments, so every peer's link
      // streams at once (one runtime copy after another would use one link at a time); without peer access
      // the runtime copies.  FTAR_LOCAL_COPY=runtime: the runtime's copy for every receive; =gather: the
      // multi-segment copy for every receive, same device included (the A/Bs, and the test of that path on
      // a one-GPU box).
      static const int copy_mode = [] {
        const char* e = getenv("FTAR_LOCAL_COPY");
        return e && !strcmp(e, "runtime") ? 0 : e && !strcmp(e, "gather") ? 2 : 1;
      }();
      ftar_status_t cst = FTAR_SUCCESS;
      if (!o.bytes) {
      } else if (copy_mode == 2 || (copy_mode == 1 && p->device != dev && hub_->can_reach(dev, p->device))) {
        per_stream_segs(gathers, o.s)->push_back({p->buf, o.buf, o.bytes});
      } else if (copy_mode == 1 && p->device == dev) {
        cst = launch_copy(p->buf, o.buf, o.bytes, o.s);
      } else if (hipMemcpyAsync(o.buf, p->buf, o.bytes, hipMemcpyDeviceToDevice, o.s) != hipSuccess) {
        set_error("local transport: hipMemcpyAsync failed", __FILE__, __LINE__);
        cst = FTAR_ERR_HIP;
      }
      if (cst != FTAR_SUCCESS) return publish(cst);
    }
    for (auto& g : gathers)
      for (size_t i = 0; i < g.second.size(); i += FTAR_MAX_K) {
        const int m = (int)std::min<size_t>(FTAR_MAX_K, g.second.size() - i);
        const ftar_status_t gst = launch_gather(g.second.data() + i, m, g.first);
        if (gst != FTAR_SUCCESS) return publish(gst);
      }
    FTAR_RETURN_IF(publish(FTAR_SUCCESS));
    // 3. the sender's stream may not move on (and overwrite the source) before the copy
    waited.clear();
    size_t i = 0;
    for (auto& o : ops) {
      if (!o.is_send) continue;
      auto& p = mine[i++];
      Ev d;
      {
        std::unique_lock<std::mutex> g(hub_->mu);
        if (!hub_->wait(g, rank_, [&] { return p->taken || !hub_->broken.empty(); })) {
          set_error("local transport: send to rank " + std::to_string(o.peer) + " never received", __FILE__,
                    __LINE__);
          return FTAR_ERR_TIMEOUT;
        }
        if (!p->taken) {
          set_error("local transport: another rank failed before receiving (" + hub_->broken + ")", __FILE__,
                    __LINE__);
          return FTAR_ERR_INTERNAL;
        }
        d = p->done;
      }
      if (!d) {
        set_error("local transport: rank " + std::to_string(o.peer) + " failed to receive", __FILE__, __LINE__);
        return FTAR_ERR_INTERNAL;
      }
      const std::pair<hipStream_t, hipEvent_t> w{o.s, *d};
      if (std::find(waited.begin(), waited.end(), w) == waited.end()) {
        FTAR_CHECK_HIP(hipStreamWaitEvent(o.s, *d, 0));
        waited.push_back(w);
      }
    }
    return FTAR_SUCCESS;
  }

  std::shared_ptr<LocalHub> hub_;
  int rank_;
  int depth_ = 0;
  std::vector<Op> ops_;
};

}  // namespace

std::unique_ptr<Transport> make_local_transport(std::shared_ptr<LocalHub> hub, int rank) {
  return std::unique_ptr<Transport>(new LocalTransport(std::move(hub), rank));
}

// ---------------------------------------------------------------------------
// caller-bootstrapped processes (ftar_comm_init_host): peer-direct only
// ---------------------------------------------------------------------------
// Point-to-point transfers are unsupported: the one-round plans run in the
// peer-direct forms (kernel loads/stores through IPC-mapped buffers), whose
// barriers and handle exchanges go through the caller's host allgather.
// (Round 1 carried an experimental host-synchronous bounce-buffer p2p here; a
// long 4-process run on one GPU stalled in it, and as no product path used it,
// it was removed.)
namespace {
class HostTransport final : public Transport {
 public:
  HostTransport(int nranks, int rank, ftar_host_allgather_fn fn, void* user)
      : nranks_(nranks), rank_(rank), fn_(fn), user_(user) {}
  ftar_status_t group_start() override { return FTAR_SUCCESS; }
  ftar_status_t send(const void*, size_t, int, hipStream_t) override { return unsupported(); }
  ftar_status_t recv(void*, size_t, int, hipStream_t) override { return unsupported(); }
  ftar_status_t group_end() override { return FTAR_SUCCESS; }
  ftar_status_t allgather(const void*, void*, size_t, int, int, hipStream_t) override { return unsupported(); }
  const char* name() const override { return "host"; }
  bool uses_ipc() const override { return true; }
  bool async_p2p() const override { return false; }
  // everything before it on s, on every rank, is complete when it returns
  ftar_status_t barrier(hipStream_t s) override {
    bool ok = true;
    FTAR_RETURN_IF(barrier_status(s, true, &ok));
    if (!ok) {
      set_error("host transport: another rank failed before this barrier", __FILE__, __LINE__);
      return FTAR_ERR_INTERNAL;
    }
    return FTAR_SUCCESS;
  }
  // a failed stream synchronisation is this rank's failure, reported to the others rather than returned
  // before the host collective (which would leave them waiting in it)
  ftar_status_t barrier_status(hipStream_t s, bool mine_ok, bool* all_ok) override {
    const hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
      set_error(std::string("host transport barrier: hipStreamSynchronize: ") + hipGetErrorString(e), __FILE__,
                __LINE__);
      mine_ok = false;
    }
    const char mine = mine_ok ? 1 : 0;
    std::vector<char> all(nranks_);
    FTAR_RETURN_IF(gather(&mine, all.data(), 1));
    *all_ok = true;
    for (char v : all) *all_ok = *all_ok && v == 1;
    return FTAR_SUCCESS;
  }
  ftar_status_t agree(const void* mine, size_t bytes, bool* same) override {
    std::vector<char> all((size_t)nranks_ * bytes);
    FTAR_RETURN_IF(gather(mine, all.data(), bytes));
    *same = true;
    for (int q = 0; q < nranks_; ++q) *same = *same && !memcmp(all.data() + (size_t)q * bytes, mine, bytes);
    return FTAR_SUCCESS;
  }
  ftar_status_t map_peers(void* mine, int rank, int nranks, std::vector<char*>* peers) override {
    if (nranks != nranks_ || rank != rank_) return FTAR_ERR_INVALID_ARG;
    IpcRef ref;
    const bool exported = ipc_export(mine, &ref) == FTAR_SUCCESS;
    std::vector<IpcRef> all(nranks);
    FTAR_RETURN_IF(gather(&ref, all.data(), sizeof ref));
    peers->assign(nranks, nullptr);
    int failed = exported ? 0 : 1;
    for (int q = 0; q < nranks; ++q)  // a failed export anywhere: nobody opens anything
      if (all[q].valid != 1) failed = 1;
    // one rank at a time opens the peers' handles (see RcclTransport::map_peers);
    // every turn ends with an agreement on the failures so far: all map or none
    std::vector<int> flags(nranks);
    for (int turn = 0; turn < nranks; ++turn) {
      for (int q = 0; q < nranks && turn == rank && !failed; ++q) {
        if (q == rank) {
          (*peers)[q] = static_cast<char*>(mine);
          continue;
        }
        if (imports_.open(all[q], &(*peers)[q]) != FTAR_SUCCESS) failed = 1;
      }
      FTAR_RETURN_IF(gather(&failed, flags.data(), sizeof failed));
      for (int f : flags) failed |= f;
    }
    if (failed) {
      unmap_peers(peers, rank);
      set_error("host transport: a rank could not map the peers' buffers", __FILE__, __LINE__);
      return FTAR_ERR_HIP;
    }
    return FTAR_SUCCESS;
  }
  void unmap_peers(std::vector<char*>* peers, int rank) override { imports_.close_all(peers, rank); }

 private:
  static ftar_status_t unsupported() {
    set_error("host transport: point-to-point transfers are unsupported (one-round plans in the peer-direct "
              "forms only)",
              __FILE__, __LINE__);
    return FTAR_ERR_UNSUPPORTED;
  }
  ftar_status_t gather(const void* mine, void* all, size_t bytes) {
    if (fn_(mine, all, bytes, user_) != 0) {
      set_error("host transport: the caller's allgather failed", __FILE__, __LINE__);
      return FTAR_ERR_INTERNAL;
    }
    return FTAR_SUCCESS;
  }
  int nranks_, rank_;
  ftar_host_allgather_fn fn_;
  void* user_;
  PeerImports imports_;
};
}  // namespace

std::unique_ptr<Transport> make_host_transport(int nranks, int rank, ftar_host_allgather_fn fn, void* user) {
  return std::unique_ptr<Transport>(new HostTransport(nranks, rank, fn, user));
}

}  // namespace ftar
