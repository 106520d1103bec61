// The C ABI of the engine (include/ftar.h): communicator bring-up and teardown, the setters and getters,
// the AllReduce entry points and the in-process group calls.  Split out of engine.cpp (round 5); no
// behaviour change.
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "engine_state.h"

using ftar::hip_ignore;

extern "C" {

ftar_status_t ftar_comm_init_rank(ftar_comm_t* comm, int nranks, ftar_unique_id_t id, int rank, int device) {
  if (!comm || nranks <= 0 || rank < 0 || rank >= nranks) return FTAR_ERR_INVALID_ARG;
  std::unique_ptr<ftar_comm> c(new ftar_comm);
  c->rank = rank;
  c->nranks = nranks;
  c->device = device;
  FTAR_CHECK_HIP(hipSetDevice(device));
  ftar_status_t st = FTAR_SUCCESS;
  c->tp = ftar::make_rccl_transport(nranks, id, rank, &st);
  if (st != FTAR_SUCCESS) return st;
  st = ftar::comm_setup(c.get());
  if (st != FTAR_SUCCESS) {
    ftar::comm_teardown(c.get());
    return st;
  }
  *comm = c.release();
  return FTAR_SUCCESS;
}

ftar_status_t ftar_comm_init_host(ftar_comm_t* comm, int nranks, int rank, int device, ftar_host_allgather_fn allgather,
                                  void* user) {
  if (!comm || !allgather || nranks <= 0 || rank < 0 || rank >= nranks) return FTAR_ERR_INVALID_ARG;
  std::unique_ptr<ftar_comm> c(new ftar_comm);
  c->rank = rank;
  c->nranks = nranks;
  c->device = device;
  c->tp = ftar::make_host_transport(nranks, rank, allgather, user);
  ftar_status_t st = ftar::comm_setup(c.get());
  if (st != FTAR_SUCCESS) {
    ftar::comm_teardown(c.get());
    return st;
  }
  *comm = c.release();
  return FTAR_SUCCESS;
}

ftar_status_t ftar_comm_init_local(ftar_comm_t* comms, int nranks, const int* devices) {
  if (!comms || nranks <= 0) return FTAR_ERR_INVALID_ARG;
  // ranks on different GPUs of this process copy straight over xGMI
  for (int a = 0; devices && a < nranks; ++a)
    for (int b = 0; b < nranks; ++b) {
      if (devices[a] == devices[b]) continue;
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, devices[a], devices[b]) == hipSuccess && can) {
        FTAR_CHECK_HIP(hipSetDevice(devices[a]));
        hipError_t e = hipDeviceEnablePeerAccess(devices[b], 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) FTAR_CHECK_HIP(e);
        (void)hipGetLastError();
      }
    }
  auto hub = ftar::make_local_hub(nranks);
  std::vector<ftar_comm*> made;
  for (int r = 0; r < nranks; ++r) {
    auto* c = new ftar_comm;
    c->rank = r;
    c->nranks = nranks;
    c->device = devices ? devices[r] : 0;
    c->tp = ftar::make_local_transport(hub, r);
    ftar_status_t st = ftar::comm_setup(c);
    if (st != FTAR_SUCCESS) {
      ftar::comm_teardown(c);
      delete c;
      for (auto* m : made) {
        ftar::comm_teardown(m);
        delete m;
      }
      return st;
    }
    made.push_back(c);
  }
  for (int r = 0; r < nranks; ++r) comms[r] = made[r];
  return FTAR_SUCCESS;
}

ftar_status_t ftar_comm_destroy(ftar_comm_t comm) {
  if (!comm) return FTAR_ERR_INVALID_ARG;
  if (ftar::comm_teardown(comm)) delete comm;  // else a stuck first contact still uses it: left behind
  return FTAR_SUCCESS;
}

ftar_status_t ftar_comm_rank(ftar_comm_t comm, int* rank) {
  if (!comm || !rank) return FTAR_ERR_INVALID_ARG;
  *rank = comm->rank;
  return FTAR_SUCCESS;
}
ftar_status_t ftar_comm_size(ftar_comm_t comm, int* size) {
  if (!comm || !size) return FTAR_ERR_INVALID_ARG;
  *size = comm->nranks;
  return FTAR_SUCCESS;
}
const char* ftar_comm_transport(ftar_comm_t comm) { return comm && comm->tp ? comm->tp->name() : ""; }

ftar_status_t ftar_comm_device(ftar_comm_t comm, int* device) {
  if (!comm || !device) return FTAR_ERR_INVALID_ARG;
  *device = comm->device;
  return FTAR_SUCCESS;
}
// Introspection for tools/rccl_order/queue_probe.cpp (not in ftar.h): the communicator's internal streams
// (comm, reduce, H2D, D2H; null where not created), so the probe can tell which of them share a hardware queue.
extern "C" ftar_status_t ftar_debug_comm_streams(ftar_comm_t comm, void** streams4) {
  if (!comm || !streams4) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  streams4[0] = comm->comm_s;
  streams4[1] = comm->red_s;
  streams4[2] = comm->h2d_s;
  streams4[3] = comm->d2h_s;
  return FTAR_SUCCESS;
}
ftar_status_t ftar_comm_set_chunk_bytes(ftar_comm_t comm, size_t bytes) {
  if (!comm) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  comm->chunk_bytes = bytes ? std::max<size_t>(256, bytes & ~size_t(255)) : 0;  // 0: the model's piece
  return FTAR_SUCCESS;
}

ftar_status_t ftar_comm_set_form(ftar_comm_t comm, int form) {
  if (!comm || form < FTAR_FORM_AUTO || form > FTAR_FORM_PEER_WRITE) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  if (!comm->tp->async_p2p() && form != FTAR_FORM_PEER_READ && form != FTAR_FORM_PEER_WRITE) {
    ftar::set_error("a host-bootstrapped communicator moves data by the peer forms only", __FILE__, __LINE__);
    return FTAR_ERR_UNSUPPORTED;
  }
  ftar::set_form(comm, form);
  return FTAR_SUCCESS;
}

ftar_status_t ftar_comm_get_form(ftar_comm_t comm, int* form) {
  if (!comm || !form) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  *form = comm->form;
  return FTAR_SUCCESS;
}

ftar_status_t ftar_comm_last_exec(ftar_comm_t comm, ftar_exec_t* out) {
  if (!comm || !out) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  *out = comm->last_exec;
  return FTAR_SUCCESS;
}
ftar_status_t ftar_comm_set_allgather(ftar_comm_t comm, ftar_allgather_t mode) {
  if (!comm || (mode != FTAR_AG_STAGES && mode != FTAR_AG_COLLECTIVE && mode != FTAR_AG_DIRECT))
    return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  comm->allgather = mode;
  comm->form = ftar::form_of(comm);
  return FTAR_SUCCESS;
}

ftar_status_t ftar_comm_set_reduce_scatter(ftar_comm_t comm, ftar_reduce_scatter_t mode) {
  if (!comm || (mode != FTAR_RS_STAGES && mode != FTAR_RS_DIRECT)) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  comm->reduce_scatter = mode;
  comm->form = ftar::form_of(comm);
  return FTAR_SUCCESS;
}

ftar_status_t ftar_comm_get_reduce_scatter(ftar_comm_t comm, ftar_reduce_scatter_t* mode) {
  if (!comm || !mode) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  *mode = static_cast<ftar_reduce_scatter_t>(comm->reduce_scatter);
  return FTAR_SUCCESS;
}

ftar_status_t ftar_comm_get_allgather(ftar_comm_t comm, ftar_allgather_t* mode) {
  if (!comm || !mode) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  *mode = static_cast<ftar_allgather_t>(comm->allgather);
  return FTAR_SUCCESS;
}

ftar_status_t ftar_comm_get_chunk_bytes(ftar_comm_t comm, size_t* bytes) {
  if (!comm || !bytes) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  *bytes = comm->chunk_bytes;
  return FTAR_SUCCESS;
}

ftar_status_t ftar_allreduce(const void* sendbuf, void* recvbuf, size_t count, ftar_dtype_t dtype, ftar_op_t op,
                             const ftar_topo_t* topo, ftar_comm_t comm, void* stream) {
  return ftar::allreduce(sendbuf, recvbuf, count, dtype, op, topo, comm, static_cast<hipStream_t>(stream));
}

ftar_status_t ftar_allreduce_host(const void* sendbuf, void* recvbuf, size_t count, ftar_dtype_t dtype, ftar_op_t op,
                                  const ftar_topo_t* topo, ftar_comm_t comm, void* stream) {
  if (!recvbuf && count) return FTAR_ERR_INVALID_ARG;
  const ftar::HostIO io{static_cast<const char*>(sendbuf ? sendbuf : recvbuf), static_cast<char*>(recvbuf)};
  return ftar::allreduce(sendbuf, recvbuf ? recvbuf : io.dst, count, dtype, op, topo, comm,
                         static_cast<hipStream_t>(stream), &io);
}

// Test hook (not in ftar.h): the transport's peer plumbing on a real
// communicator -- map a fresh allocation (IPC handle exchange), barrier on the
// comm stream, unmap.  On a 1-rank RCCL communicator this runs every RCCL and
// IPC call of the peer path except opening another rank's handle.
ftar_status_t ftar_debug_peer_selftest(ftar_comm_t comm) {
  if (!comm) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  FTAR_CHECK_HIP(hipSetDevice(comm->device));
  void* buf = nullptr;
  FTAR_CHECK_HIP(hipMalloc(&buf, 1 << 20));
  std::vector<char*> peers;
  ftar_status_t st = comm->tp->map_peers(buf, comm->rank, comm->nranks, &peers);
  if (st == FTAR_SUCCESS && (peers.size() != (size_t)comm->nranks || peers[comm->rank] != buf)) st = FTAR_ERR_INTERNAL;
  if (st == FTAR_SUCCESS) st = comm->tp->barrier(comm->comm_s);
  if (st == FTAR_SUCCESS && hipStreamSynchronize(comm->comm_s) != hipSuccess) st = FTAR_ERR_HIP;
  comm->tp->unmap_peers(&peers, comm->rank);
  hip_ignore(hipFree(buf));
  return st;
}

ftar_status_t ftar_comm_set_peer_direct(ftar_comm_t comm, int mode) {
  if (!comm || mode < FTAR_PEER_OFF || mode > FTAR_PEER_WRITE) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  comm->peer_direct = mode;
  comm->form = ftar::form_of(comm);
  return FTAR_SUCCESS;
}

// Test/tuning hook (not in ftar.h): peer-form copies nontemporal (nt) or not,
// fold through the LDS-staged kernel (lds) or the register kernel.
ftar_status_t ftar_debug_set_peer_tuning(ftar_comm_t comm, int nt, int lds) {
  if (!comm) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  comm->peer_nt = nt != 0;
  comm->peer_lds = lds != 0;
  return FTAR_SUCCESS;
}
// Test/tuning hook (not in ftar.h): the peer forms' cross-GPU copies by the DMA engines.
ftar_status_t ftar_debug_set_peer_wg_cap(ftar_comm_t comm, size_t wg_per_segment) {
  if (!comm) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  comm->peer_wg_cap = wg_per_segment;
  return FTAR_SUCCESS;
}

// RCCL registration of the comm's scratch buffer (FTAR_RCCL_REGISTER); off drops it at once.
ftar_status_t ftar_debug_set_rccl_register(ftar_comm_t comm, int on) {
  if (!comm) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  comm->rccl_reg = on != 0;
  if (!comm->rccl_reg && comm->scratch_rccl) {
    FTAR_CHECK_HIP(hipSetDevice(comm->device));
    FTAR_CHECK_HIP(hipStreamSynchronize(comm->comm_s));
    FTAR_CHECK_HIP(hipStreamSynchronize(comm->red_s));
    comm->tp->rccl_deregister(comm->scratch_rccl);
    comm->scratch_rccl = nullptr;
  }
  return FTAR_SUCCESS;
}

ftar_status_t ftar_debug_set_peer_dma(ftar_comm_t comm, int dma) {
  if (!comm) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  comm->peer_dma = dma != 0;
  return FTAR_SUCCESS;
}

ftar_status_t ftar_comm_get_peer_direct(ftar_comm_t comm, int* mode) {
  if (!comm || !mode) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  *mode = comm->peer_direct;
  return FTAR_SUCCESS;
}

ftar_status_t ftar_comm_register(ftar_comm_t comm, void* buf, size_t bytes, int* reg) {
  if (!comm || !buf || !bytes || !reg) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  FTAR_CHECK_HIP(hipSetDevice(comm->device));
  ftar_comm::Reg r{static_cast<char*>(buf), bytes, {}};
  FTAR_RETURN_IF(comm->tp->map_peers(buf, comm->rank, comm->nranks, &r.peers));
  r.rccl = comm->tp->rccl_register(buf, bytes);  // RCCL's own registration too (local; nullptr if refused)
  *reg = comm->next_reg++;
  comm->regs.emplace(*reg, std::move(r));
  return FTAR_SUCCESS;
}

ftar_status_t ftar_comm_deregister(ftar_comm_t comm, int reg) {
  if (!comm) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  auto it = comm->regs.find(reg);
  if (it == comm->regs.end()) return FTAR_ERR_INVALID_ARG;
  FTAR_CHECK_HIP(hipSetDevice(comm->device));
  FTAR_CHECK_HIP(hipStreamSynchronize(comm->comm_s));  // its last call ended in a barrier: no peer touches it
  FTAR_CHECK_HIP(hipStreamSynchronize(comm->red_s));
  comm->tp->unmap_peers(&it->second.peers, comm->rank);
  comm->tp->rccl_deregister(it->second.rccl);
  comm->regs.erase(it);
  return FTAR_SUCCESS;
}

ftar_status_t ftar_comm_set_phase_timing(ftar_comm_t comm, int enable) {
  if (!comm) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  comm->phase_timing = enable != 0;
  comm->nmarks = 0;
  return FTAR_SUCCESS;
}

long ftar_comm_phase_json(ftar_comm_t comm, char* buf, size_t buflen) {
  if (!comm) return -FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  std::string j = "[";
  if (comm->nmarks) {
    if (hipSetDevice(comm->device) != hipSuccess) return -FTAR_ERR_HIP;
    for (size_t i = 0; i < comm->nmarks; ++i)
      if (hipEventSynchronize(comm->tev[i]) != hipSuccess) return -FTAR_ERR_HIP;
    for (size_t i = 0; i < comm->nmarks; ++i) {
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, comm->tev[0], comm->tev[i]) != hipSuccess) return -FTAR_ERR_HIP;
      char item[160];
      snprintf(item, sizeof item, "%s[\"%s\", %.4f]", i ? ", " : "", comm->tnames[i].c_str(), (double)ms);
      j += item;
    }
  }
  j += "]";
  if (buf && buflen) {
    const size_t m = std::min(buflen - 1, j.size());
    memcpy(buf, j.data(), m);
    buf[m] = 0;
  }
  return (long)j.size();
}

ftar_status_t ftar_xgmi_probe(ftar_comm_t comm, size_t bytes_per_peer, int iters, double* gbps, int n) {
  if (!comm || !gbps || n <= 0 || iters <= 0 || bytes_per_peer == 0) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  FTAR_CHECK_HIP(hipSetDevice(comm->device));
  return ftar::xgmi_probe(comm, bytes_per_peer, iters, gbps, n, 0);
}

// Test/tuning hook (not in ftar.h): the probe with at most wg_per_peer
// workgroups of 256 threads per peer segment -- how many CUs saturate xGMI.
ftar_status_t ftar_debug_xgmi_probe_cap(ftar_comm_t comm, size_t bytes_per_peer, int iters, size_t wg_per_peer,
                                        double* gbps, int n) {
  if (!comm || !gbps || n <= 0 || iters <= 0 || bytes_per_peer == 0) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  FTAR_CHECK_HIP(hipSetDevice(comm->device));
  return ftar::xgmi_probe(comm, bytes_per_peer, iters, gbps, n, wg_per_peer);
}

// Test hook (not in ftar.h): rank `peer`'s exchange buffer as this process maps it (peer == own rank: its
// own) and its size; null and 0 before the first peer-form call.  The full-size host-comm tests poison their
// own buffer between cases and compare every rank's view of every mapping page by page.
ftar_status_t ftar_debug_exchange_buffer(ftar_comm_t comm, int peer, void** ptr, size_t* bytes) {
  if (!comm || !ptr || !bytes || peer < 0 || peer >= comm->nranks) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  *ptr = nullptr;
  *bytes = 0;
  if (!comm->xbuf || comm->xpeers.size() != (size_t)comm->nranks) return FTAR_SUCCESS;
  *ptr = peer == comm->rank ? comm->xbuf : comm->xpeers[(size_t)peer];
  *bytes = comm->xbuf_bytes;
  return FTAR_SUCCESS;
}

// Test hook (not in ftar.h): the gather records of piece `piece` of the last host-path call made
// under FTAR_DEBUG_HOST_GATHER_LOG=1 -- host_rec: 4 words per workgroup in host memory, dev_rec: per workgroup
// id the number of times it ran and the XCDs it ran on, 2 words in device memory (reduce_impl.h
// gather_logged_kernel) -- and info[4 + 2 * FTAR_MAX_K] = {pieces
// logged, grid, segments, tile bytes, each segment's destination offset in the exchange buffer, its bytes}.
// Read them only after the call completed.
ftar_status_t ftar_debug_gather_log(ftar_comm_t comm, size_t piece, const unsigned** host_rec,
                                    const unsigned** dev_rec, size_t* info) {
  if (!comm || !host_rec || !dev_rec || !info) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  const auto& L = comm->glog;
  std::fill(info, info + 4 + 2 * FTAR_MAX_K, size_t(0));
  info[0] = L.pieces.size();
  *host_rec = nullptr;
  *dev_rec = nullptr;
  if (piece >= L.pieces.size()) return FTAR_SUCCESS;
  const auto& p = L.pieces[piece];
  *host_rec = L.host + 4 * p.first;
  *dev_rec = L.dev + 2 * p.first;
  info[1] = p.geom.grid;
  info[2] = p.geom.nsegs;
  info[3] = p.geom.tile_bytes;
  for (unsigned j = 0; j < p.geom.nsegs; ++j) {
    info[4 + j] = p.off[j];
    info[4 + FTAR_MAX_K + j] = p.bytes[j];
  }
  return FTAR_SUCCESS;
}

ftar_status_t ftar_comm_set_reduce_cus(ftar_comm_t comm, int cus) {
  if (!comm) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  FTAR_CHECK_HIP(hipSetDevice(comm->device));
  return ftar::set_reduce_cus(comm, cus);
}

ftar_status_t ftar_comm_get_reduce_cus(ftar_comm_t comm, int* cus) {
  if (!comm || !cus) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  *cus = comm->reduce_cus;
  return FTAR_SUCCESS;
}

ftar_status_t ftar_comm_set_host_chunk_bytes(ftar_comm_t comm, size_t bytes) {
  if (!comm) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  comm->host_chunk_bytes = bytes ? std::max<size_t>(256, bytes & ~size_t(255)) : ftar::kDefaultHostChunkBytes;
  return FTAR_SUCCESS;
}

ftar_status_t ftar_comm_get_host_chunk_bytes(ftar_comm_t comm, size_t* bytes) {
  if (!comm || !bytes) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  *bytes = comm->host_chunk_bytes;
  return FTAR_SUCCESS;
}

ftar_status_t ftar_rccl_allreduce(const void* sendbuf, void* recvbuf, size_t count, ftar_dtype_t dtype, ftar_op_t op,
                                  ftar_comm_t comm, void* stream) {
  if (!comm || !recvbuf) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  FTAR_CHECK_HIP(hipSetDevice(comm->device));
  return comm->tp->native_allreduce(sendbuf == recvbuf ? nullptr : sendbuf, recvbuf, count, dtype, op,
                                    static_cast<hipStream_t>(stream));
}

namespace {
// Host threads for the ranks of the in-process group calls, kept from call to call instead of one
// std::thread per rank per call (their start and join sat inside every call's time).  The ranks of a call
// meet in the transport, so they must all run at once: every job is handed to a worker that is free at
// that moment, and a call that finds fewer free workers than ranks starts more (the pool only grows; its
// workers wait on a condition variable between calls).  Leaked on purpose -- the workers are detached.
class RankPool {
 public:
  static RankPool& get() {
    static std::atomic<RankPool*> pool{nullptr};
    RankPool* p = pool.load();
    if (!p || p->pid_ != getpid()) {  // first use, or a forked child (the parent's workers are not here)
      RankPool* fresh = new RankPool;
      if (pool.compare_exchange_strong(p, fresh)) return *fresh;
      delete fresh;  // another thread installed one first
      return *pool.load();
    }
    return *p;
  }
  // fn(0) ... fn(n - 1), all at once on pool workers; returns when every one has returned
  void run(int n, const std::function<void(int)>& fn) {
    Latch done{n};
    {
      std::lock_guard<std::mutex> g(mu_);
      const int take = std::min(free_, n);
      free_ -= take;
      for (int i = take; i < n; ++i) std::thread([this] { work(); }).detach();
      for (int r = 0; r < n; ++r) q_.push_back({&fn, r, &done});
    }
    cv_.notify_all();
    std::unique_lock<std::mutex> lk(done.mu);
    done.cv.wait(lk, [&] { return done.left == 0; });
  }

 private:
  struct Latch {
    int left;
    std::mutex mu;
    std::condition_variable cv;
  };
  struct Job {
    const std::function<void(int)>* fn;
    int rank;
    Latch* done;
  };
  // a worker is started for a job already counted against it, and counts itself free again only once
  // its job has returned: so every queued job has a worker that is not busy with anything else.  It
  // counts itself free before it reports the job done, so the caller's next call finds it free.
  void work() {
    for (;;) {
      Job j;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return !q_.empty(); });
        j = q_.front();
        q_.pop_front();
      }
      (*j.fn)(j.rank);
      {
        std::lock_guard<std::mutex> g(mu_);
        ++free_;
      }
      std::lock_guard<std::mutex> g(j.done->mu);
      if (--j.done->left == 0) j.done->cv.notify_all();
    }
  }
  const pid_t pid_ = getpid();
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Job> q_;
  int free_ = 0;
};

ftar_status_t run_group(const void* const* sendbufs, void* const* recvbufs, size_t count, ftar_dtype_t dtype,
                        ftar_op_t op, const ftar_topo_t* topo, ftar_comm_t* comms, int nranks,
                        void* const* streams, bool host) {
  if (!recvbufs || !comms || nranks <= 0) return FTAR_ERR_INVALID_ARG;
  std::vector<ftar_status_t> st(nranks, FTAR_SUCCESS);
  std::vector<std::string> why(nranks);
  // Capturing streams (the caller's capture stream for every rank): the ranks' threads take turns issuing
  // (Transport::capture_enter), and nobody synchronises; the caller ends the capture.
  bool capturing = false;
  if (streams && streams[0]) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    FTAR_CHECK_HIP(hipSetDevice(comms[0]->device));
    FTAR_CHECK_HIP(hipStreamIsCapturing(static_cast<hipStream_t>(streams[0]), &cs));
    capturing = cs != hipStreamCaptureStatusNone;
  }
  // Under capture every rank's call goes on the caller's capture stream itself.  A stream forked per rank
  // from the capture makes HIP's hipStreamEndCapture recurse without end at every P probed, 7.0 and 7.2 alike,
  // even when ftar funnels the ranks onto one of those streams (tools/capture/depth_probe.sh,
  // profiles/r04/capture_depth_probe.log): refused here rather than crashing the caller at its end of capture.
  if (capturing)
    for (int r = 1; r < nranks; ++r)
      if (streams[r] != streams[0]) {
        ftar::set_error("ftar_allreduce_group under stream capture: pass the capture stream itself for every rank "
                        "(streams forked per rank make hipStreamEndCapture recurse without end)",
                        __FILE__, __LINE__);
        return FTAR_ERR_UNSUPPORTED;
      }
  auto rank_call = [&](int r) {
    hipStream_t s = streams ? static_cast<hipStream_t>(streams[r]) : nullptr;
    const void* sb = sendbufs ? sendbufs[r] : nullptr;
    if (capturing) comms[r]->tp->capture_enter();
    st[r] = host ? ftar_allreduce_host(sb, recvbufs[r], count, dtype, op, topo, comms[r], s)
                 : ftar::allreduce(sb, recvbufs[r], count, dtype, op, topo, comms[r], s);
    if (capturing) comms[r]->tp->capture_leave();
    // device buffers: the call returns once every rank's work is enqueued on its stream (stream order, as
    // ftar_allreduce and RCCL's group calls); host buffers: once they hold the result
    if (host && !capturing && st[r] == FTAR_SUCCESS && hipSetDevice(comms[r]->device) == hipSuccess &&
        hipStreamSynchronize(s) != hipSuccess)
      st[r] = FTAR_ERR_HIP;
    if (st[r] != FTAR_SUCCESS) why[r] = ftar::last_error();  // the error text is per thread
  };
  RankPool::get().run(nranks, rank_call);
  for (int r = 0; r < nranks; ++r)
    if (st[r] != FTAR_SUCCESS) {
      ftar::set_error("rank " + std::to_string(r) + ": " + why[r], __FILE__, __LINE__);  // to the caller's thread
      return st[r];
    }
  return FTAR_SUCCESS;
}
}  // namespace

// Test hook (not in ftar.h): `rounds` calls of the group thread pool, each of n jobs that meet at a
// rendezvous the way a group call's ranks meet in the transport -- a job left waiting for a worker would
// hang it, so it waits at most a second.  Returns how many rendezvous were complete, out of rounds.
int ftar_debug_rank_pool(int n, int rounds) {
  if (n <= 0 || rounds <= 0) return -1;
  int complete = 0;
  for (int i = 0; i < rounds; ++i) {
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    std::atomic<int> met{0};
    RankPool::get().run(n, [&](int) {
      std::unique_lock<std::mutex> lk(mu);
      if (++arrived == n) cv.notify_all();
      if (cv.wait_for(lk, std::chrono::seconds(1), [&] { return arrived == n; })) ++met;
    });
    complete += met.load() == n;
  }
  return complete;
}

ftar_status_t ftar_allreduce_group(const void* const* sendbufs, void* const* recvbufs, size_t count,
                                   ftar_dtype_t dtype, ftar_op_t op, const ftar_topo_t* topo, ftar_comm_t* comms,
                                   int nranks, void* const* streams) {
  return run_group(sendbufs, recvbufs, count, dtype, op, topo, comms, nranks, streams, false);
}

ftar_status_t ftar_allreduce_host_group(const void* const* sendbufs, void* const* recvbufs, size_t count,
                                        ftar_dtype_t dtype, ftar_op_t op, const ftar_topo_t* topo,
                                        ftar_comm_t* comms, int nranks, void* const* streams) {
  return run_group(sendbufs, recvbufs, count, dtype, op, topo, comms, nranks, streams, true);
}

}  // extern "C"
