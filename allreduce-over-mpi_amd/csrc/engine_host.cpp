// Host buffers on a host-bootstrapped communicator (engine_state.h): the read form piece by piece, H2D /
// exchange / D2H overlapped (the MPI drop-in's `ipc` transport).  Split out of engine.cpp (round 5); no
// behaviour change.
#include <algorithm>
#include <cstring>

#include "engine_state.h"

using ftar::hip_ignore;

namespace ftar {

constexpr size_t kMaxHostPeerPieces = 1024;  // peer_allreduce_host: pieces per call (a host barrier each)

// Elements per piece of peer_allreduce_host.  Auto: at least 8 pieces per block down to 4 MiB (2 ranks
// on one GPU, 64 MiB buckets: 4 MiB pieces 16.5 GB/s vs 12.6 with two 16 MiB pieces;
// profiles/r02/s4/host_ipc/), else the p2p host path's rule; every piece costs a host barrier and two
// events, so at most kMaxHostPeerPieces pieces per call.
size_t host_peer_piece(const ftar_comm* c, size_t split, size_t esz) {
  const size_t chunk_bytes =
      c->host_chunk_bytes
          ? c->host_chunk_bytes
          : std::max(split * esz / 64, std::min<size_t>(16u << 20, std::max<size_t>(4u << 20, split * esz / 8)));
  const size_t floor_elems = (split + kMaxHostPeerPieces - 1) / kMaxHostPeerPieces;
  return std::max<size_t>({64, (chunk_bytes / esz) & ~size_t(63), (floor_elems + 63) & ~size_t(63)});
}

// FTAR_DEBUG_HOST_GATHER_LOG (diagnostic): the gather of piece k with one record per workgroup
// (launch_gather_logged), read back by ftar_debug_gather_log.  The records are cleared at the call's first
// logged gather (`first`), after the host waited for the comm stream (no gather of an earlier call still
// writes them); room for m pieces of that gather's grid.  Always the copy kernel (peer_dma is not consulted).
static ftar_status_t log_gather(ftar_comm* c, const std::vector<Segment>& segs, const char* X, bool first, size_t m) {
  ftar_comm::GatherLog& L = c->glog;
  const GatherGeom g = gather_geometry(segs.data(), (int)segs.size(), c->peer_wg_cap);
  if (first) {
    FTAR_CHECK_HIP(hipStreamSynchronize(c->comm_s));
    const size_t need = m * (size_t)g.grid;
    if (need > L.cap) {
      if (L.host) FTAR_CHECK_HIP(hipHostFree(L.host));
      if (L.dev) FTAR_CHECK_HIP(hipFree(L.dev));
      L.host = nullptr;
      L.dev = nullptr;
      L.cap = 0;
      FTAR_CHECK_HIP(hipHostMalloc(reinterpret_cast<void**>(&L.host), need * 4 * sizeof(unsigned),
                                   hipHostMallocCoherent));
      FTAR_CHECK_HIP(hipMalloc(reinterpret_cast<void**>(&L.dev), need * 2 * sizeof(unsigned)));
      L.cap = need;
    }
    memset(L.host, 0, L.cap * 4 * sizeof(unsigned));
    FTAR_CHECK_HIP(hipMemsetAsync(L.dev, 0, L.cap * 2 * sizeof(unsigned), c->comm_s));
    L.pieces.clear();
  }
  ftar_comm::GatherLog::Piece p{};
  p.first = L.pieces.empty() ? 0 : L.pieces.back().first + L.pieces.back().geom.grid;
  p.geom = g;
  if (p.first + g.grid > L.cap) return FTAR_ERR_INTERNAL;
  size_t j = 0;
  for (const Segment& s : segs)
    if (s.bytes) {
      p.off[j] = (size_t)(static_cast<const char*>(s.dst) - X);
      p.bytes[j++] = s.bytes;
    }
  FTAR_RETURN_IF(launch_gather_logged(segs.data(), (int)segs.size(), c->comm_s, c->peer_nt, c->peer_wg_cap,
                                      L.host + 4 * p.first, L.dev + 2 * p.first, L.cap - p.first));
  L.pieces.push_back(p);
  return FTAR_SUCCESS;
}

// Host buffers on a communicator without point-to-point transfers (ftar_comm_init_host: the MPI
// drop-in's `ipc` transport), the read form piece by piece, as the p2p host path pipelines its
// stages.  Piece k is elements [k*chunk, (k+1)*chunk) of every block.
//   * every piece goes H2D straight into the exchange buffer X on its own stream, kHostPeerLookahead
//     pieces ahead of the fold that needs it, so the copy engines run ahead while the host waits at
//     the barriers (no staging buffer, no copy-in pass);
//   * once every rank's piece k is in (a barrier), the fold of my block's piece k reads the peers'
//     copies from their X over xGMI and writes my X in place (the plan's fold: same bits);
//   * once every rank's fold of piece k is done (the next barrier, which also says piece k+1 is in
//     everywhere), the other owners' final pieces are pulled into my X at their offsets, and piece
//     k of the whole bucket goes D2H on its own stream while later pieces come in.
// A peer reads my X only at its own block (fold) and at my block (gather), and I overwrite my X
// only at my block (fold, before anyone gathers it) and at the others' blocks (gather, after every
// fold of that piece), so pieces never conflict.  The barriers synchronise the host: m pieces take
// m + 2 barriers, the last so that no peer still reads my X when the next call's H2D refills it.
ftar_status_t peer_allreduce_host(const HostIO& io, size_t count, ftar_dtype_t dt, ftar_op_t op, const Plan& plan,
                                  ftar_comm* c, hipStream_t stream) {
  const size_t esz = dtype_size(dt), bytes = count * esz;
  FTAR_RETURN_IF(ensure_xbuf(c, bytes));  // collective, before the first barrier
  Transport* tp = c->tp.get();
  char* X = static_cast<char*>(c->xbuf);
  const std::vector<char*>& Xq = c->xpeers;
  const Stage& rs = plan.stages[0];
  const Stage& ag = plan.stages[1];
  const size_t P = (size_t)c->nranks, split = plan.split;
  const size_t chunk = host_peer_piece(c, split, esz);
  const size_t m = std::max<size_t>(1, (split + chunk - 1) / chunk);
  // The D2H pieces go on the reduce stream, which this path leaves idle (its folds and gathers run on
  // the comm stream): on 4 hardware queues the H2D and D2H streams of a host-bootstrapped communicator
  // share one queue (tools/rccl_order/queue_probe --ipc --host-call, profiles/r05/queues/), and copies
  // on one queue run in issue order, so the two directions never overlapped.
  // Diagnostics (tools/host_comm_stress.py): FTAR_DEBUG_HOST_D2H_STREAM=1 puts the D2H pieces back on the
  // host D2H stream, FTAR_DEBUG_HOST_LOOKAHEAD=n issues the H2D pieces n ahead (large: all up front, as
  // round 5's one c4_host_read mismatch ran)
  static const bool d2h_own = getenv("FTAR_DEBUG_HOST_D2H_STREAM") && atoi(getenv("FTAR_DEBUG_HOST_D2H_STREAM"));
  static const size_t lookahead =
      getenv("FTAR_DEBUG_HOST_LOOKAHEAD") ? (size_t)atol(getenv("FTAR_DEBUG_HOST_LOOKAHEAD")) : kHostPeerLookahead;
  hipStream_t d2h = d2h_own ? c->d2h_s : c->red_s;
  // FTAR_DEBUG_HOST_GATHER_FENCE (diagnostic): 1 an empty kernel after each gather, before the event the D2H
  // waits on; 2 the gather's workgroups end with a system-scope release; 3 the gather with temporal stores
  static const int gather_fence =
      getenv("FTAR_DEBUG_HOST_GATHER_FENCE") ? atoi(getenv("FTAR_DEBUG_HOST_GATHER_FENCE")) : 0;
  // FTAR_DEBUG_HOST_D2H_ORDER=host (diagnostic): the D2H of piece k is issued only once the host has seen
  // the gather of piece k complete (after the next barrier) instead of waiting for its event on the device
  static const bool d2h_host_order =
      getenv("FTAR_DEBUG_HOST_D2H_ORDER") && !strcmp(getenv("FTAR_DEBUG_HOST_D2H_ORDER"), "host");
  // FTAR_DEBUG_HOST_GATHER_LOG=1 (diagnostic): each gather workgroup leaves a record of where and when it
  // ran (launch_gather_logged; ftar_debug_gather_log reads them after the call)
  static const bool gather_log = getenv("FTAR_DEBUG_HOST_GATHER_LOG") && atoi(getenv("FTAR_DEBUG_HOST_GATHER_LOG"));
  // Every rank goes through all m + 2 barriers whatever fails locally: `st` keeps this rank's first
  // failure, the work after it is skipped, and each barrier tells every rank whether any rank failed,
  // so all of them leave the call at the same barrier instead of some waiting in the next.
  ftar_status_t st = grow_events(c, 5 + 2 * m);
  hipEvent_t* ev = c->events.data();
  auto ev_h = [&](size_t k) { return c->events[5 + 2 * k]; };      // piece k is in my X
  auto ev_g = [&](size_t k) { return c->events[5 + 2 * k + 1]; };  // piece k is final in my X
  auto for_piece = [&](size_t k, auto&& fn) -> ftar_status_t {  // piece k of every block, clipped
    for (size_t b = 0; b < P; ++b) {
      const size_t lo = b * split + k * chunk, end = std::min(count, (b + 1) * split);
      if (lo < end) FTAR_RETURN_IF(fn(lo, std::min(chunk, end - lo)));
    }
    return FTAR_SUCCESS;
  };
  // Order matters when the copy streams share a hardware queue with the comm stream (HIP's 4 queues
  // per process): commands of a shared queue run in issue order, and a barrier waits for the
  // comm stream.  So every H2D piece is issued after the fold commands of an earlier piece (never all
  // up front: the first barrier then waited for the whole bucket), and the D2H of piece k after the
  // fold of piece k + 1 (else that fold, and the barrier after it, waited for the D2H).
  size_t h2d_issued = 0;
  auto issue_h2d = [&](size_t upto) -> ftar_status_t {  // pieces [h2d_issued, upto]
    for (; h2d_issued <= upto && h2d_issued < m; ++h2d_issued) {
      const size_t k = h2d_issued;
      FTAR_RETURN_IF(for_piece(k, [&](size_t lo, size_t n) -> ftar_status_t {
        FTAR_CHECK_HIP(hipMemcpyAsync(X + lo * esz, io.src + lo * esz, n * esz, hipMemcpyHostToDevice, c->h2d_s));
        return FTAR_SUCCESS;
      }));
      FTAR_CHECK_HIP(hipEventRecord(ev_h(k), c->h2d_s));
      FTAR_RETURN_IF(mark(c, "h2d " + std::to_string(k) + " done", c->h2d_s));
    }
    return FTAR_SUCCESS;
  };
  auto issue_d2h = [&](size_t k) -> ftar_status_t {  // piece k of the whole bucket, once it is final here
    FTAR_CHECK_HIP(hipStreamWaitEvent(d2h, ev_g(k), 0));
    FTAR_RETURN_IF(mark(c, "d2h " + std::to_string(k) + " start", d2h));
    FTAR_RETURN_IF(for_piece(k, [&](size_t lo2, size_t n) -> ftar_status_t {
      FTAR_CHECK_HIP(hipMemcpyAsync(io.dst + lo2 * esz, X + lo2 * esz, n * esz, hipMemcpyDeviceToHost, d2h));
      return FTAR_SUCCESS;
    }));
    return mark(c, "d2h " + std::to_string(k) + " done", d2h);
  };
  auto work = [&](auto&& fn) {
    if (st == FTAR_SUCCESS) st = fn();
  };
  // a failed call leaves only after its copies stopped touching the caller's host buffers: H2D reads of
  // io.src and D2H writes of io.dst may still be in flight on their streams
  auto leave = [&]() -> ftar_status_t {
    for (hipStream_t s : {c->h2d_s, d2h, c->comm_s})
      if (s) hip_ignore(hipStreamSynchronize(s));
    return st;
  };
  auto sync = [&]() -> bool {  // a barrier; false: some rank failed, leave the call
    bool all_ok = true;
    const ftar_status_t b = tp->barrier_status(c->comm_s, st == FTAR_SUCCESS, &all_ok);
    if (b != FTAR_SUCCESS) {  // the host collective itself failed: nothing left to agree with
      if (st == FTAR_SUCCESS) st = b;
      return false;
    }
    if (!all_ok && st == FTAR_SUCCESS) {
      set_error("peer_allreduce_host: another rank failed", __FILE__, __LINE__);
      st = FTAR_ERR_INTERNAL;
    }
    return all_ok;
  };
  work([&]() -> ftar_status_t {
    ev = c->events.data();
    FTAR_CHECK_HIP(hipEventRecord(ev[0], stream));
    for (hipStream_t s : {c->comm_s, c->h2d_s, d2h}) FTAR_CHECK_HIP(hipStreamWaitEvent(s, ev[0], 0));
    c->nmarks = 0;
    FTAR_RETURN_IF(mark(c, "start", c->comm_s));
    FTAR_RETURN_IF(issue_h2d(lookahead));
    FTAR_CHECK_HIP(hipStreamWaitEvent(c->comm_s, ev_h(0), 0));
    return FTAR_SUCCESS;
  });
  if (!sync()) return leave();  // piece 0 is in everywhere
  work([&] { return mark(c, "piece 0 in", c->comm_s); });
  std::vector<Segment> segs;
  bool logged = false;                    // FTAR_DEBUG_HOST_GATHER_LOG: this call logged a gather
  if (gather_log) c->glog.pieces.clear();  // no records of an earlier call stay readable
  for (size_t k = 0; k < m; ++k) {
    const size_t lo = k * chunk;
    work([&]() -> ftar_status_t {
      // phase timing (ftar_comm_set_phase_timing): every hand-off of the piece has a mark on its stream, the
      // happens-before check of tools/host_order_check.py --marks
      FTAR_RETURN_IF(mark(c, "fold " + std::to_string(k) + " start", c->comm_s));
      for (const ReduceItem& r : rs.reduces)
        FTAR_RETURN_IF(peer_fold(
            r, plan, dt, op, X + (r.off + lo) * esz, c->comm_s, c->peer_lds,
            [&](int q, size_t off) -> const void* { return (q < 0 ? X : Xq[q]) + off * esz; }, lo, chunk));
      FTAR_RETURN_IF(mark(c, "fold " + std::to_string(k) + " done", c->comm_s));
      if (k + 1 < m) FTAR_CHECK_HIP(hipStreamWaitEvent(c->comm_s, ev_h(k + 1), 0));
      FTAR_RETURN_IF(issue_h2d(k + 1 + lookahead));  // after this fold's commands (see above)
      if (k > 0 && !d2h_host_order) FTAR_RETURN_IF(issue_d2h(k - 1));  // likewise
      return FTAR_SUCCESS;
    });
    if (!sync()) return leave();  // piece k folded everywhere (and piece k+1 in)
    work([&]() -> ftar_status_t {
      if (k > 0 && d2h_host_order) FTAR_RETURN_IF(issue_d2h(k - 1));
      FTAR_RETURN_IF(mark(c, "gather " + std::to_string(k) + " start", c->comm_s));
      segs.clear();
      for (const Transfer& x : ag.recvs)
        if (x.len > lo)
          segs.push_back(
              {Xq[x.peer] + (x.off + lo) * esz, X + (x.off + lo) * esz, std::min(chunk, x.len - lo) * esz});
      if (!segs.empty()) {
        if (gather_log) {
          FTAR_RETURN_IF(log_gather(c, segs, X, !logged, m));
          logged = true;
        } else if (gather_fence == 2 || gather_fence == 3) {
          FTAR_RETURN_IF(launch_gather(segs.data(), (int)segs.size(), c->comm_s, gather_fence == 2 && c->peer_nt,
                                       c->peer_wg_cap, gather_fence == 2));
        } else {
          FTAR_RETURN_IF(peer_copy(c, segs));
        }
        if (gather_fence == 1) FTAR_RETURN_IF(launch_noop(c->comm_s));
      }
      FTAR_RETURN_IF(mark(c, "gather " + std::to_string(k) + " done", c->comm_s));
      FTAR_CHECK_HIP(hipEventRecord(ev_g(k), c->comm_s));
      return k + 1 == m && !d2h_host_order ? issue_d2h(k) : FTAR_SUCCESS;  // the others after the next fold
    });
  }
  work([&]() -> ftar_status_t {
    if (!d2h_host_order) return FTAR_SUCCESS;
    FTAR_CHECK_HIP(hipStreamSynchronize(c->comm_s));
    return issue_d2h(m - 1);
  });
  work([&]() -> ftar_status_t {
    FTAR_RETURN_IF(mark(c, "pieces folded and gathered", c->comm_s));
    // the last barrier also waits for my D2H pieces: after it nothing of this call reads my X, my own
    // copies included, so a peer's next call may write into it at once (the write form scatters into
    // the peers' X before its first barrier)
    FTAR_CHECK_HIP(hipEventRecord(ev[2], d2h));
    FTAR_CHECK_HIP(hipStreamWaitEvent(c->comm_s, ev[2], 0));
    return FTAR_SUCCESS;
  });
  if (!sync()) return leave();  // no peer reads my X after the call, and my D2H is done
  if (st != FTAR_SUCCESS) return leave();
  FTAR_RETURN_IF(mark(c, "barrier", c->comm_s));
  FTAR_RETURN_IF(tp->before_join());
  FTAR_CHECK_HIP(hipEventRecord(ev[1], c->comm_s));
  FTAR_CHECK_HIP(hipEventRecord(ev[3], c->h2d_s));
  for (int i = 1; i <= 3; ++i) FTAR_CHECK_HIP(hipStreamWaitEvent(stream, ev[i], 0));
  return FTAR_SUCCESS;
}

}  // namespace ftar
