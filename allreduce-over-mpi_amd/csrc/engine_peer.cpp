// The peer-direct forms (engine_state.h): one-round plans moved by kernel loads or stores through
// IPC-mapped exchange buffers over xGMI, registered buffers in place, and the xGMI probe.  Split out of
// engine.cpp (round 5); no behaviour change.
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <map>
#include <thread>

#include "engine_state.h"

using ftar::hip_ignore;

namespace ftar {

// ---------------------------------------------------------------------------
// Peer-direct execution of a one-round plan (ring or tree, direct forms): no
// RCCL data movement, no scratch pass.  Kernels move the blocks over xGMI
// through IPC-mapped exchange buffers X (grow-only, comm-owned), and the
// plan's own fold (operand order, nested shape, bf16 rounding) runs
// unchanged, so the bits are the plan's.  Two forms:
//
//  READ (pull)   in -> X | barrier | fold my block reading every rank's copy
//                from X_q, into X | barrier | gather every owner's block from
//                X_q -> recvbuf | barrier (X stays intact until all have read)
//  WRITE (push)  scatter: my copy of q's block -> X_q.slot[me], all peers in
//                one launch | barrier | fold my block from in + X.slot[*]
//                into recvbuf | push it -> X_q.final[my block] | barrier |
//                X.final[other blocks] -> recvbuf
//                Two barriers: call i's scatter lands after every rank passed
//                call i-1's second barrier (its fold is done), and its pushes
//                after every rank's call i-1 copy-out (first barrier of i).
//
// The barriers are stream-ordered (Transport::barrier), nothing spins on the
// device.  Cross-GPU visibility rests on kernel-boundary release/acquire.
// ---------------------------------------------------------------------------
bool peer_eligible(const Plan& plan) {
  if (plan.stages.size() != 2 || plan.allgather != FTAR_AG_DIRECT || plan.nranks > FTAR_MAX_K) return false;
  const Stage& rs = plan.stages[0];
  const Stage& ag = plan.stages[1];
  if (rs.reduces.size() > 1) return false;
  std::vector<int> seen_s(plan.nranks, 0), seen_r(plan.nranks, 0), seen_a(plan.nranks, 0);
  for (const Transfer& x : rs.sends)  // one block per peer each way (the write form's slot = sender)
    if (x.buf != BUF_SRC || x.len > plan.split || seen_s[x.peer]++) return false;
  for (const Transfer& x : rs.recvs)
    if (x.buf != BUF_SCRATCH || seen_r[x.peer]++) return false;
  for (const ReduceItem& r : rs.reduces)
    for (const Operand& o : r.srcs)
      if (o.buf == BUF_DST) return false;
  for (const Transfer& x : ag.recvs)
    if (x.buf != BUF_DST || seen_a[x.peer]++) return false;
  for (const Transfer& x : ag.sends)
    if (x.buf != BUF_DST) return false;
  return ag.reduces.empty();
}

// grow-only exchange buffer, exported and mapped by every rank (collective)
//
// Under the HIP runtime torch bundles (7.0), a fresh allocation whose address
// range was an IPC mapping a moment before can fail hipIpcGetMemHandle
// (alloc_exportable sets such allocations aside), and an import can map the
// wrong memory after regrowth (ipc_import verifies every mapping against the
// owner's stamped token).  Nothing here returns before map_peers: every rank
// must reach the exchange; a failed rank publishes an invalid reference and
// all ranks fail, and retry, together.
ftar_status_t refuse_growth_under_capture(const ftar_comm* c, const char* what) {
  if (!c->capturing) return FTAR_SUCCESS;
  set_error(std::string(what) + " would grow during stream capture: make one call of the same shape before "
                                "capturing (growth allocates and synchronises)",
            __FILE__, __LINE__);
  return FTAR_ERR_UNSUPPORTED;
}

ftar_status_t ensure_xbuf(ftar_comm* c, size_t bytes) {
  if (bytes <= c->xbuf_bytes && !c->xpeers.empty()) return FTAR_SUCCESS;
  FTAR_RETURN_IF(refuse_growth_under_capture(c, "the exchange buffer"));
  Transport* tp = c->tp.get();
  FTAR_CHECK_HIP(hipStreamSynchronize(c->comm_s));  // the last barrier: no peer still touches the old X
  FTAR_CHECK_HIP(hipStreamSynchronize(c->red_s));
  const size_t need = std::max(bytes, c->xbuf_bytes);
  trace("rank %d: exchange buffer %zu -> >= %zu bytes", c->rank, c->xbuf_bytes, need);
  // The new X is allocated, stamped and mapped while the old X and the old
  // mappings are still alive (a fresh allocation or import landing on an
  // address range just released is where the runtime went wrong); a mapping
  // that fails verification on any rank is retried by all, the failed
  // allocation kept until the end so the next one lands elsewhere.
  std::vector<void*> failed;
  std::vector<char*> peers;
  void* fresh = nullptr;
  size_t got = 0;
  ftar_status_t st = FTAR_ERR_HIP;
  for (int attempt = 0; attempt < 3 && st != FTAR_SUCCESS; ++attempt) {
    fresh = nullptr;
    got = 0;
    if (alloc_exportable(need, tp->uses_ipc(), &fresh, &got) == FTAR_SUCCESS && tp->uses_ipc() &&
        stamp_token(fresh) != FTAR_SUCCESS) {
      hip_ignore(hipFree(fresh));
      fresh = nullptr;
    }
    st = tp->map_peers(fresh, c->rank, c->nranks, &peers);
    trace("rank %d: exchange buffer at %p, map peers -> %d", c->rank, fresh, (int)st);
    if (st != FTAR_SUCCESS && fresh) failed.push_back(fresh);
  }
  tp->unmap_peers(&c->xpeers, c->rank);
  if (c->xbuf) {
    forget_token(c->xbuf);
    hip_ignore(hipFree(c->xbuf));
  }
  c->xbuf = nullptr;
  c->xbuf_bytes = 0;
  for (void* f : failed) {
    forget_token(f);
    hip_ignore(hipFree(f));
  }
  if (st != FTAR_SUCCESS) {
    if (fresh && std::find(failed.begin(), failed.end(), fresh) == failed.end()) hip_ignore(hipFree(fresh));
    return st;
  }
  c->xbuf = fresh;
  c->xbuf_bytes = got;
  c->xpeers.swap(peers);
  return FTAR_SUCCESS;
}

// the plan's fold of my block with operand i read from where(i); elements
// [lo, lo + len) of the block only (a piece of it, host mode), dst at element lo
ftar_status_t peer_fold(const ReduceItem& r, const Plan& plan, ftar_dtype_t dt, ftar_op_t op, void* dst,
                        hipStream_t s, bool lds, const OperandAt& where, size_t lo, size_t len) {
  std::map<size_t, int> slot_peer;  // scratch slot -> the rank that would have sent it
  for (const Transfer& x : plan.stages[0].recvs) slot_peer[x.off] = x.peer;
  std::vector<const void*> srcs;
  for (const Operand& o : r.srcs) {
    if (o.buf == BUF_SRC) {
      srcs.push_back(where(-1, o.off + lo));
    } else {
      auto it = slot_peer.find(o.off);
      if (it == slot_peer.end()) return FTAR_ERR_INTERNAL;
      srcs.push_back(where(it->second, r.off + lo));
    }
  }
  if (lo >= r.len) return FTAR_SUCCESS;
  return launch_reduce(srcs.data(), (int)srcs.size(), dst, std::min(len, r.len - lo), dt, op, s, r.round_each,
                       r.shape.data(), (int)r.shape.size(), lds);
}

namespace {
// the registration holding [p, p+bytes), or null
const ftar_comm::Reg* find_reg(const ftar_comm* c, const void* p, size_t bytes) {
  const char* q = static_cast<const char*>(p);
  for (const auto& r : c->regs)
    if (q >= r.second.ptr && q + bytes <= r.second.ptr + r.second.bytes) return &r.second;
  return nullptr;
}
// rank `peer`'s buffer at the same offset into its registration as p into mine
char* reg_peer(const ftar_comm::Reg* r, const void* p, int peer) {
  return r->peers[peer] + (static_cast<const char*>(p) - r->ptr);
}
}  // namespace

// the peer forms' cross-GPU copies: one copy-kernel launch over every segment (every link at once), or with
// peer_dma one DMA copy per segment, each on its own stream, all joined back into comm_s
ftar_status_t peer_copy(ftar_comm* c, const std::vector<Segment>& segs) {
  if (!c->peer_dma) return launch_gather(segs.data(), (int)segs.size(), c->comm_s, c->peer_nt, c->peer_wg_cap);
  if (c->serial) {  // a serial capture: the DMA copies in turn on the one stream
    for (const Segment& g : segs)
      if (g.bytes) FTAR_CHECK_HIP(hipMemcpyAsync(g.dst, g.src, g.bytes, hipMemcpyDeviceToDevice, c->comm_s));
    return FTAR_SUCCESS;
  }
  if (!c->dma_fork) FTAR_CHECK_HIP(hipEventCreateWithFlags(&c->dma_fork, hipEventDisableTiming));
  while (c->dma_s.size() < segs.size()) {
    hipStream_t t;
    hipEvent_t e;
    FTAR_CHECK_HIP(hipStreamCreateWithFlags(&t, hipStreamNonBlocking));
    FTAR_CHECK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c->dma_s.push_back(t);
    c->dma_ev.push_back(e);
  }
  FTAR_CHECK_HIP(hipEventRecord(c->dma_fork, c->comm_s));
  for (size_t i = 0; i < segs.size(); ++i) {
    if (!segs[i].bytes) continue;
    FTAR_CHECK_HIP(hipStreamWaitEvent(c->dma_s[i], c->dma_fork, 0));
    FTAR_CHECK_HIP(hipMemcpyAsync(segs[i].dst, segs[i].src, segs[i].bytes, hipMemcpyDeviceToDevice, c->dma_s[i]));
    FTAR_CHECK_HIP(hipEventRecord(c->dma_ev[i], c->dma_s[i]));
    FTAR_CHECK_HIP(hipStreamWaitEvent(c->comm_s, c->dma_ev[i], 0));
  }
  return FTAR_SUCCESS;
}

ftar_status_t peer_allreduce(const void* sendbuf, void* recvbuf, size_t count, ftar_dtype_t dt, ftar_op_t op,
                             const Plan& plan, ftar_comm* c, hipStream_t stream, int mode) {
  const size_t esz = dtype_size(dt), bytes = count * esz;
  const bool write = mode == FTAR_PEER_WRITE;
  const size_t slot_bytes = plan.split * esz, final_at = (size_t)plan.nranks * slot_bytes;
  char* out = static_cast<char*>(recvbuf);
  const char* in = static_cast<const char*>(sendbuf ? sendbuf : recvbuf);
  // registered buffers (every rank's, at the same offsets): no local pass --
  // read: peers' inputs and outputs are read in place; write: final blocks are
  // pushed straight into the peers' outputs
  const ftar_comm::Reg* rin = find_reg(c, in, bytes);
  const ftar_comm::Reg* rout = find_reg(c, out, bytes);
  const bool zc = write ? rout != nullptr : (rin != nullptr && rout != nullptr);
  FTAR_RETURN_IF(ensure_xbuf(c, write ? final_at + (zc ? 0 : bytes) : (zc ? 256 : bytes)));
  Transport* tp = c->tp.get();
  char* X = static_cast<char*>(c->xbuf);
  const std::vector<char*>& Xq = c->xpeers;
  const Stage& rs = plan.stages[0];
  const Stage& ag = plan.stages[1];
  hipEvent_t* ev = c->events.data();
  FTAR_CHECK_HIP(hipEventRecord(ev[0], stream));
  FTAR_CHECK_HIP(hipStreamWaitEvent(c->comm_s, ev[0], 0));
  c->nmarks = 0;
  FTAR_RETURN_IF(mark(c, "start", c->comm_s));
  std::vector<Segment> segs;
  if (!write && zc) {
    FTAR_RETURN_IF(tp->barrier(c->comm_s));  // every rank's input is ready
    FTAR_RETURN_IF(mark(c, "barrier", c->comm_s));
    for (const ReduceItem& r : rs.reduces)
      FTAR_RETURN_IF(peer_fold(r, plan, dt, op, out + r.off * esz, c->comm_s, c->peer_lds, [&](int q, size_t off) -> const void* {
        return q < 0 ? in + off * esz : reg_peer(rin, in, q) + off * esz;  // that rank's input, in place
      }));
    FTAR_RETURN_IF(mark(c, "fold (remote reads)", c->comm_s));
    FTAR_RETURN_IF(tp->barrier(c->comm_s));
    FTAR_RETURN_IF(mark(c, "barrier", c->comm_s));
    for (const Transfer& x : ag.recvs)
      segs.push_back({reg_peer(rout, out, x.peer) + x.off * esz, out + x.off * esz, x.len * esz});
    FTAR_RETURN_IF(peer_copy(c, segs));
    FTAR_RETURN_IF(mark(c, "gather (remote reads)", c->comm_s));
    FTAR_RETURN_IF(tp->barrier(c->comm_s));  // no peer reads my buffers after the call
    FTAR_RETURN_IF(mark(c, "barrier", c->comm_s));
  } else if (!write) {
    const Segment whole{in, X, bytes};
    FTAR_RETURN_IF(c->peer_nt ? launch_copy(in, X, bytes, c->comm_s) : launch_gather(&whole, 1, c->comm_s, false));
    FTAR_RETURN_IF(mark(c, "copy-in", c->comm_s));
    FTAR_RETURN_IF(tp->barrier(c->comm_s));
    FTAR_RETURN_IF(mark(c, "barrier", c->comm_s));
    for (const ReduceItem& r : rs.reduces)
      FTAR_RETURN_IF(peer_fold(r, plan, dt, op, X + r.off * esz, c->comm_s, c->peer_lds, [&](int q, size_t off) -> const void* {
        return q < 0 ? X + off * esz : Xq[q] + off * esz;  // that rank's copy of this block
      }));
    FTAR_RETURN_IF(mark(c, "fold (remote reads)", c->comm_s));
    FTAR_RETURN_IF(tp->barrier(c->comm_s));
    FTAR_RETURN_IF(mark(c, "barrier", c->comm_s));
    // all-gather: every owner's final block from its exchange buffer, one launch
    for (const ReduceItem& r : rs.reduces) segs.push_back({X + r.off * esz, out + r.off * esz, r.len * esz});
    for (const Transfer& x : ag.recvs) segs.push_back({Xq[x.peer] + x.off * esz, out + x.off * esz, x.len * esz});
    FTAR_RETURN_IF(peer_copy(c, segs));
    FTAR_RETURN_IF(mark(c, "gather (remote reads)", c->comm_s));
    FTAR_RETURN_IF(tp->barrier(c->comm_s));
    FTAR_RETURN_IF(mark(c, "barrier", c->comm_s));
  } else {
    // scatter my copy of every peer's block into its slot for me, all links at once
    for (const Transfer& x : rs.sends)
      segs.push_back({in + x.off * esz, Xq[x.peer] + (size_t)c->rank * slot_bytes, x.len * esz});
    FTAR_RETURN_IF(peer_copy(c, segs));
    FTAR_RETURN_IF(mark(c, "scatter (remote writes)", c->comm_s));
    FTAR_RETURN_IF(tp->barrier(c->comm_s));
    FTAR_RETURN_IF(mark(c, "barrier", c->comm_s));
    for (const ReduceItem& r : rs.reduces)
      FTAR_RETURN_IF(peer_fold(r, plan, dt, op, out + r.off * esz, c->comm_s, c->peer_lds, [&](int q, size_t off) -> const void* {
        return q < 0 ? in + off * esz : X + (size_t)q * slot_bytes;  // rank q's copy, pushed into slot q
      }));
    FTAR_RETURN_IF(mark(c, "fold (local)", c->comm_s));
    segs.clear();  // my final block into every peer's final area, or straight into its registered output
    for (const Transfer& x : ag.sends)
      segs.push_back({out + x.off * esz, (zc ? reg_peer(rout, out, x.peer) : Xq[x.peer] + final_at) + x.off * esz,
                      x.len * esz});
    FTAR_RETURN_IF(peer_copy(c, segs));
    FTAR_RETURN_IF(mark(c, "push (remote writes)", c->comm_s));
    FTAR_RETURN_IF(tp->barrier(c->comm_s));
    FTAR_RETURN_IF(mark(c, "barrier", c->comm_s));
    if (!zc) {
      segs.clear();
      for (const Transfer& x : ag.recvs) segs.push_back({X + final_at + x.off * esz, out + x.off * esz, x.len * esz});
      // test hook (tests/rccl_loopback_child.py write_race): this rank enqueues its copy-out late, as a slow
      // host would, so a peer already in its next call writes into this exchange buffer meanwhile
      static const long late_us = getenv("FTAR_DEBUG_PEER_LATE_US") ? atol(getenv("FTAR_DEBUG_PEER_LATE_US")) : 0;
      if (late_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(late_us));
      if (c->peer_nt) {
        for (const Segment& g : segs) FTAR_RETURN_IF(launch_copy(g.src, g.dst, g.bytes, c->comm_s));
      } else {
        FTAR_RETURN_IF(launch_gather(segs.data(), (int)segs.size(), c->comm_s, false));
      }
      FTAR_RETURN_IF(mark(c, "copy-out", c->comm_s));
      // no peer may scatter its next call into my X before my copy-out has read it: a call whose slot area
      // covers this call's final area would overwrite it (tools/asan/engine_stress rccl found it; test:
      // test_peer_write_waits_for_every_copy_out)
      FTAR_RETURN_IF(tp->barrier(c->comm_s));
      FTAR_RETURN_IF(mark(c, "barrier", c->comm_s));
    }
  }
  FTAR_RETURN_IF(tp->before_join());
  FTAR_CHECK_HIP(hipEventRecord(ev[1], c->comm_s));
  FTAR_CHECK_HIP(hipStreamWaitEvent(stream, ev[1], 0));
  return FTAR_SUCCESS;
}

// xGMI probe (diagnostic, collective): every rank runs the same copy pattern
// at the same time between barriers, timed with events on the comm stream.
ftar_status_t xgmi_probe(ftar_comm* c, size_t bytes, int iters, double* out, int nout, size_t max_wg_per_seg) {
  const int P = c->nranks, me = c->rank;
  FTAR_RETURN_IF(ensure_xbuf(c, 2 * (size_t)P * bytes));  // P send slots + P receive slots
  Transport* tp = c->tp.get();
  char* X = static_cast<char*>(c->xbuf);
  const std::vector<char*>& Xq = c->xpeers;
  auto send_slot = [&](char* base, int q) { return base + (size_t)q * bytes; };
  auto recv_slot = [&](char* base, int q) { return base + (size_t)(P + q) * bytes; };
  hipEvent_t e0, e1;
  FTAR_CHECK_HIP(hipEventCreate(&e0));
  FTAR_CHECK_HIP(hipEventCreate(&e1));
  ftar_status_t st = FTAR_SUCCESS;
  const int nxt = (me + 1) % P, prv = (me + P - 1) % P;
  // DMA modes: one hipMemcpyAsync per peer, each on its own stream (forked from and joined back into the
  // comm stream), so the copy engines rather than CUs move the bytes
  std::vector<hipStream_t> ds;
  std::vector<hipEvent_t> dj;
  hipEvent_t fork = nullptr;
  auto dma = [&](const std::vector<Segment>& segs) -> ftar_status_t {
    if (!fork) FTAR_CHECK_HIP(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    while (ds.size() < segs.size()) {
      hipStream_t t;
      hipEvent_t e;
      FTAR_CHECK_HIP(hipStreamCreateWithFlags(&t, hipStreamNonBlocking));
      FTAR_CHECK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      ds.push_back(t);
      dj.push_back(e);
    }
    FTAR_CHECK_HIP(hipEventRecord(fork, c->comm_s));
    for (size_t i = 0; i < segs.size(); ++i) {
      FTAR_CHECK_HIP(hipStreamWaitEvent(ds[i], fork, 0));
      FTAR_CHECK_HIP(hipMemcpyAsync(segs[i].dst, segs[i].src, segs[i].bytes, hipMemcpyDeviceToDevice, ds[i]));
      FTAR_CHECK_HIP(hipEventRecord(dj[i], ds[i]));
      FTAR_CHECK_HIP(hipStreamWaitEvent(c->comm_s, dj[i], 0));
    }
    return FTAR_SUCCESS;
  };
  // 0 local copy | 1 read from one peer | 2 read from all | 3 write to one | 4 write to all (copy kernels)
  // 5 read from all | 6 write to all (DMA engines)
  for (int mode = 0; mode < std::min(nout, 7) && st == FTAR_SUCCESS; ++mode) {
    std::vector<Segment> segs;
    if (mode == 0) segs.push_back({send_slot(X, 0), recv_slot(X, 0), bytes});
    if (mode == 1 && P > 1) segs.push_back({send_slot(Xq[nxt], me), recv_slot(X, nxt), bytes});
    if (mode == 3 && P > 1) segs.push_back({send_slot(X, prv), recv_slot(Xq[prv], me), bytes});
    for (int q = 0; q < P; ++q) {
      if (q == me) continue;
      if (mode == 2 || mode == 5) segs.push_back({send_slot(Xq[q], me), recv_slot(X, q), bytes});
      if (mode == 4 || mode == 6) segs.push_back({send_slot(X, q), recv_slot(Xq[q], me), bytes});
    }
    out[mode] = 0.0;
    if (segs.empty()) continue;
    auto copy = [&]() {
      return mode >= 5 ? dma(segs) : launch_gather(segs.data(), (int)segs.size(), c->comm_s, true, max_wg_per_seg);
    };
    if ((st = copy()) != FTAR_SUCCESS) break;  // warm
    if ((st = tp->barrier(c->comm_s)) != FTAR_SUCCESS) break;
    if (hipEventRecord(e0, c->comm_s) != hipSuccess) st = FTAR_ERR_HIP;
    for (int i = 0; i < iters && st == FTAR_SUCCESS; ++i) st = copy();
    if (st == FTAR_SUCCESS && hipEventRecord(e1, c->comm_s) != hipSuccess) st = FTAR_ERR_HIP;
    if (st == FTAR_SUCCESS) st = tp->barrier(c->comm_s);
    if (st == FTAR_SUCCESS && hipStreamSynchronize(c->comm_s) != hipSuccess) st = FTAR_ERR_HIP;
    float ms = 0.f;
    if (st == FTAR_SUCCESS && hipEventElapsedTime(&ms, e0, e1) != hipSuccess) st = FTAR_ERR_HIP;
    if (st == FTAR_SUCCESS && ms > 0.f) out[mode] = (double)segs.size() * bytes * iters / (ms * 1e-3) / 1e9;
  }
  hip_ignore(hipStreamSynchronize(c->comm_s));
  for (hipStream_t t : ds) hip_ignore(hipStreamDestroy(t));
  for (hipEvent_t e : dj) hip_ignore(hipEventDestroy(e));
  if (fork) hip_ignore(hipEventDestroy(fork));
  hip_ignore(hipEventDestroy(e0));
  hip_ignore(hipEventDestroy(e1));
  return st;
}

}  // namespace ftar
