// FlexTree AllReduce engine: runs a rank's plan on two HIP streams.
//
// Reference execution (mpi_mod.hpp:1550-1644, :1689-1715): per stage post all
// Isend/Irecv, MPI_Waitall the receives, reduce on 14 OpenMP threads,
// MPI_Waitall the sends, MPI_Barrier — no overlap between communication and
// reduction, a global barrier every stage, host buffers.
//
// Here (device-resident, nothing blocks the host):
//   comm stream : the stage's transfers, cut into pieces of `chunk` elements
//                 (piece c of every block of the stage = one p2p group);
//   reduce stream: the reduce kernel for piece c starts as soon as piece c of
//                 the stage's receives has landed (event), while piece c+1 is
//                 still on the wire;
//   cross-stage : piece c of stage s+1's transfers waits only for piece c of
//                 the latest reducing stage (what it sends, or the scratch it
//                 overwrites two stages later, depends on nothing else);
//   scratch     : compact, two halves alternating per stage, grow-only, HBM.
// The caller's stream is joined at entry and at exit with events, so the call
// is stream-ordered like any other HIP operation.
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <cstdio>
#include <initializer_list>
#include <cstdint>
#include <map>
#include <mutex>
#include <thread>

#include "engine_state.h"

using ftar::hip_ignore;


namespace ftar {

namespace {
// Host mode pieces (0 = auto): 16 MiB per block, at least split/64 (bounds the
// number of copies for huge buckets).  4 MiB device->host copies run at only
// ~33 GB/s; larger pieces lengthen the pipeline's fill and drain (one piece of
// every block each).  16 MiB was the best or near-best size in every sweep
// (profiles/r01/host/): 8 pieces per block at P = 8 x 1 GiB.
size_t auto_host_chunk(size_t split_bytes) { return std::max<size_t>(16u << 20, split_bytes / 64); }
}  // namespace

// phase timing: one timing event per boundary, on the stream that reaches it
ftar_status_t mark(ftar_comm* c, const std::string& name, hipStream_t s) {
  if (!c->phase_timing) return FTAR_SUCCESS;
  if (c->nmarks == c->tev.size()) {
    hipEvent_t e;
    FTAR_CHECK_HIP(hipEventCreate(&e));
    c->tev.push_back(e);
    c->tnames.emplace_back();
  }
  c->tnames[c->nmarks] = name;
  FTAR_CHECK_HIP(hipEventRecord(c->tev[c->nmarks++], s));
  return FTAR_SUCCESS;
}

ftar_status_t grow_events(ftar_comm* c, size_t n) {
  if (c->capturing) {  // a fresh set for this captured call; the uncaptured set stays as it is
    for (hipEvent_t e : c->events) c->captured_events.push_back(e);
    c->events.clear();
  }
  while (c->events.size() < n) {
    hipEvent_t e;
    FTAR_CHECK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c->events.push_back(e);
  }
  return FTAR_SUCCESS;
}

// The reduce stream on `cus` of the device's CUs (0 or >= all: every CU), so
// the transport's own kernels on the comm stream (RCCL's p2p kernels, the
// local transport's copies) always find free CUs while a piece's fold runs:
// the one-shot reduce grids otherwise fill every CU.  The CUs kept are spread
// evenly over the mask (CU i is kept iff floor((i+1)*cus/N) > floor(i*cus/N)),
// so every XCD keeps its share whichever way the mask bits map to XCDs.
// hipExtStreamCreateWithCUMask makes a blocking stream (it synchronises with
// the legacy NULL stream) on a hardware queue of its own, the price of the knob.
// Refused on RCCL communicators (Transport::masked_reduce_stream_ok): two runs
// of the RCCL stress driver stalled ranks inside the first call after the knob
// moved from 0 to a CU share (profiles/r04/stress_soak/).
ftar_status_t set_reduce_cus(ftar_comm* c, int cus) {
  int total = 0;
  FTAR_CHECK_HIP(hipDeviceGetAttribute(&total, hipDeviceAttributeMultiprocessorCount, c->device));
  if (cus <= 0 || cus >= total) cus = 0;
  if (cus && c->tp && !c->tp->masked_reduce_stream_ok()) {
    set_error("the reduce stream cannot be CU-masked on a " + std::string(c->tp->name()) +
                  " communicator (ftar_comm_set_reduce_cus / FTAR_REDUCE_CUS): a masked stream is a blocking "
                  "stream on a hardware queue of its own, and over RCCL it stalled ranks (DESIGN §5.1); "
                  "0 (every CU) is the only value accepted there",
              __FILE__, __LINE__);
    return FTAR_ERR_UNSUPPORTED;
  }
  if (cus == c->reduce_cus && c->red_s) return FTAR_SUCCESS;
  hipStream_t fresh = nullptr;
  if (cus == 0) {
    FTAR_CHECK_HIP(hipStreamCreateWithFlags(&fresh, hipStreamNonBlocking));
  } else {
    std::vector<uint32_t> mask((size_t)(total + 31) / 32, 0u);
    for (int i = 0; i < total; ++i)
      if ((long)(i + 1) * cus / total > (long)i * cus / total) mask[(size_t)i / 32] |= 1u << (i % 32);
    FTAR_CHECK_HIP(hipExtStreamCreateWithCUMask(&fresh, (uint32_t)mask.size(), mask.data()));
  }
  if (c->red_s) {
    hip_ignore(hipStreamSynchronize(c->red_s));
    hip_ignore(hipStreamDestroy(c->red_s));
  }
  c->red_s = fresh;
  c->reduce_cus = cus;
  trace("rank %d: reduce stream on %d of %d CUs", c->rank, cus ? cus : total, total);
  return FTAR_SUCCESS;
}

// The form the explicit settings describe (ftar_form_t), or -2 for a mix no form names.
int form_of(const ftar_comm* c) {
  if (c->peer_direct == FTAR_PEER_READ) return FTAR_FORM_PEER_READ;
  if (c->peer_direct == FTAR_PEER_WRITE) return FTAR_FORM_PEER_WRITE;
  if (c->reduce_scatter == FTAR_RS_STAGES) return c->allgather == FTAR_AG_STAGES ? FTAR_FORM_STAGES : -2;
  if (c->allgather == FTAR_AG_DIRECT) return FTAR_FORM_DIRECT;
  return c->allgather == FTAR_AG_COLLECTIVE ? FTAR_FORM_COLLECTIVE : -2;
}

// "auto" | "direct" | "stages" | "collective" | "peer-read" | "peer-write"; -3 = none of them
int form_from_name(const std::string& m) {
  if (m == "auto" || m.empty()) return FTAR_FORM_AUTO;
  if (m == "direct") return FTAR_FORM_DIRECT;
  if (m == "stages") return FTAR_FORM_STAGES;
  if (m == "collective") return FTAR_FORM_COLLECTIVE;
  if (m == "peer-read" || m == "read") return FTAR_FORM_PEER_READ;
  if (m == "peer-write" || m == "write") return FTAR_FORM_PEER_WRITE;
  return -3;
}

// The settings of one form (the engine's three knobs): all-gather, reduce-scatter, peer mode.
void form_settings(int form, int* ag, int* rs, int* peer) {
  *ag = form == FTAR_FORM_STAGES ? FTAR_AG_STAGES : form == FTAR_FORM_COLLECTIVE ? FTAR_AG_COLLECTIVE : FTAR_AG_DIRECT;
  *rs = form == FTAR_FORM_STAGES ? FTAR_RS_STAGES : FTAR_RS_DIRECT;
  *peer = form == FTAR_FORM_PEER_READ ? FTAR_PEER_READ : form == FTAR_FORM_PEER_WRITE ? FTAR_PEER_WRITE : FTAR_PEER_OFF;
}

void set_form(ftar_comm* c, int form) {
  c->form = form;
  if (form >= FTAR_FORM_DIRECT) form_settings(form, &c->allgather, &c->reduce_scatter, &c->peer_direct);
  else if (form == FTAR_FORM_AUTO) c->peer_direct = FTAR_PEER_OFF;
}

// the host-buffer path's copy streams, created at the first host-buffer call (see comm_setup_local)
// FTAR_DEBUG_HOST_COPY_PRIORITY=1 (diagnostic, tools/host_comm_stress.py): both at the highest priority,
// which the runtime puts on hardware queues of their own -- the configuration of round 5's one
// c4_host_read mismatch
ftar_status_t ensure_host_streams(ftar_comm* c) {
  static const bool prio = getenv("FTAR_DEBUG_HOST_COPY_PRIORITY") && atoi(getenv("FTAR_DEBUG_HOST_COPY_PRIORITY"));
  for (hipStream_t* s : {&c->h2d_s, &c->d2h_s}) {
    if (*s) continue;
    if (prio) {
      int least = 0, greatest = 0;
      FTAR_CHECK_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
      FTAR_CHECK_HIP(hipStreamCreateWithPriority(s, hipStreamNonBlocking, greatest));
    } else {
      FTAR_CHECK_HIP(hipStreamCreateWithFlags(s, hipStreamNonBlocking));
    }
  }
  return FTAR_SUCCESS;
}

ftar_status_t agree_settings(ftar_comm* c, bool failed = false);

namespace {
// the local part of a communicator's bring-up: streams, events, settings from the environment
ftar_status_t comm_setup_local(ftar_comm* c) {
  FTAR_RETURN_IF(cost_file_status());  // a calibration file that does not parse fails loudly, on every rank
  FTAR_CHECK_HIP(hipSetDevice(c->device));
  FTAR_CHECK_HIP(hipStreamCreateWithFlags(&c->comm_s, hipStreamNonBlocking));
  if (const char* rc = getenv("FTAR_REDUCE_CUS")) FTAR_RETURN_IF(set_reduce_cus(c, atoi(rc)));
  else FTAR_CHECK_HIP(hipStreamCreateWithFlags(&c->red_s, hipStreamNonBlocking));
  // the H2D / D2H streams exist only once a host-buffer call needs them (ensure_host_streams): a process
  // has 4 hardware queues by default and streams beyond that share them (tools/rccl_order/queue_probe), so a
  // device-resident user keeps the comm and reduce streams on queues of their own
  FTAR_CHECK_HIP(hipEventCreateWithFlags(&c->done_ev, hipEventDisableTiming));
  if (const char* pd = getenv("FTAR_PEER_DIRECT")) {
    const std::string m(pd);
    c->peer_direct = m == "write" ? FTAR_PEER_WRITE : m == "read" ? FTAR_PEER_READ
                     : std::max(0, std::min(2, atoi(pd)));
  }
  if (const char* hp = getenv("FTAR_HOST_PEER_PIPELINE")) c->host_peer_pipeline = atoi(hp) != 0;
  if (const char* rr = getenv("FTAR_RCCL_REGISTER")) c->rccl_reg = atoi(rr) != 0;
  const char* hcb = getenv("FTAR_HOST_CHUNK_BYTES");
  c->host_chunk_bytes = hcb ? strtoull(hcb, nullptr, 0) : kDefaultHostChunkBytes;
  if (c->host_chunk_bytes && c->host_chunk_bytes < 256) c->host_chunk_bytes = 256;
  if (const char* rs = getenv("FTAR_REDUCE_SCATTER"))
    c->reduce_scatter = std::string(rs) == "stages" ? FTAR_RS_STAGES : FTAR_RS_DIRECT;
  if (const char* ag = getenv("FTAR_ALLGATHER")) {
    const std::string m(ag);
    c->allgather = m == "stages" ? FTAR_AG_STAGES : m == "collective" ? FTAR_AG_COLLECTIVE : FTAR_AG_DIRECT;
  }
  // any explicit data-movement setting fixes the form; FTAR_FORM names one (or "auto") outright
  if (getenv("FTAR_PEER_DIRECT") || getenv("FTAR_REDUCE_SCATTER") || getenv("FTAR_ALLGATHER")) c->form = form_of(c);
  if (const char* fm = getenv("FTAR_FORM")) {
    const int f = form_from_name(fm);
    if (f == -3) {
      set_error(std::string("FTAR_FORM=") + fm + ": expected auto, direct, stages, collective, peer-read or peer-write",
                __FILE__, __LINE__);
      return FTAR_ERR_INVALID_ARG;
    }
    set_form(c, f);
  }
  if (!c->tp->async_p2p()) c->form = form_of(c);  // a host-bootstrapped communicator keeps its peer form
  const char* cb = getenv("FTAR_CHUNK_BYTES");
  const size_t cbv = cb ? strtoull(cb, nullptr, 0) : 0;
  c->chunk_bytes = cbv ? std::max<size_t>(256, cbv & ~size_t(255)) : 0;
  return FTAR_SUCCESS;
}
}  // namespace

// A host-bootstrapped communicator compares its settings at bring-up, and a rank whose local bring-up
// failed still takes part in that host collective, flagging its failure, so no peer is left waiting in it
// (ADVICE r3); an RCCL one compares them at its first call (first_contact), so a rank whose RCCL bring-up
// failed leaves no peer waiting in a collective inside ftar_comm_init_rank.
ftar_status_t comm_setup(ftar_comm* c) {
  ftar_status_t st = comm_setup_local(c);
  if (!c->tp->async_p2p()) {
    const std::string local_err = st == FTAR_SUCCESS ? "" : last_error();
    const ftar_status_t ag = agree_settings(c, st != FTAR_SUCCESS);
    if (st != FTAR_SUCCESS) set_error(local_err, __FILE__, __LINE__);
    else st = ag;
    if (st == FTAR_SUCCESS) c->settings_agreed = true;
  }
  return st;
}

// The environment-derived settings that shape the messages every rank posts (piece sizes, data-movement
// forms) and the topology choice (FT_TOPO / FT_LONELY, the cost model and its constants) must be alike on
// every rank: a rank pieced differently from its peers posts transfers they do not match.  Compared once
// (collective: at bring-up, or an RCCL communicator's first call), so a mismatched launch fails every rank
// instead of hanging a call.
// Setters (ftar_comm_set_*, ftar_cost_set_params) must likewise be called alike, as RCCL's own
// configuration must.
ftar_status_t agree_settings(ftar_comm* c, bool failed) {
  auto h = [](const char* v) {  // FNV-1a of an environment string ("" = unset)
    uint64_t x = 1469598103934665603ull;
    for (const char* p = v ? v : ""; *p; ++p) x = (x ^ (unsigned char)*p) * 1099511628211ull;
    return x;
  };
  ftar_cost_params_t k;
  ftar_cost_get(&k);
  uint64_t cfg[10 + sizeof k / 8] = {(uint64_t)c->chunk_bytes, (uint64_t)c->host_chunk_bytes,
                                     (uint64_t)c->peer_direct, (uint64_t)c->host_peer_pipeline,
                                     (uint64_t)c->reduce_scatter, (uint64_t)c->allgather, (uint64_t)(int64_t)c->form,
                                     h(getenv("FT_TOPO")), h(getenv("FT_LONELY")), h(getenv("FTAR_COST_MODEL"))};
  static_assert(sizeof k % 8 == 0, "cost params are doubles");
  memcpy(&cfg[10], &k, sizeof k);
  if (failed) cfg[0] = ~uint64_t(0);  // this rank's bring-up failed: no peer can match it
  bool same = true;
  FTAR_RETURN_IF(c->tp->agree(cfg, sizeof cfg, &same));
  if (failed) return FTAR_ERR_INTERNAL;
  if (!same) {
    set_error("another rank's bring-up failed, or the ranks disagree on FTAR_CHUNK_BYTES / FTAR_HOST_CHUNK_BYTES / "
              "FTAR_PEER_DIRECT / FTAR_HOST_PEER_PIPELINE / FTAR_REDUCE_SCATTER / FTAR_ALLGATHER / FTAR_FORM / FT_TOPO / FT_LONELY / "
              "the cost model or its constants: launch every rank with the same environment",
              __FILE__, __LINE__);
    return FTAR_ERR_INVALID_ARG;
  }
  return FTAR_SUCCESS;
}

// A communicator's first contact: the settings agreement, then (RCCL) one byte each way with every peer so
// that RCCL's lazy p2p connection handshakes happen here and no later call's ncclGroupEnd blocks on one.
// Where the transport may block the host in it (RCCL), it runs on a helper thread that the caller waits for
// with a deadline, FTAR_FIRST_CONTACT_TIMEOUT_S (default 600 s; 0 = no helper, no deadline): a peer that
// never shows up, or a transport stuck at its first transfer, then fails the call with FTAR_ERR_TIMEOUT
// instead of hanging it (bench.py's RCCL preflight relies on it), and the communicator is
// marked broken -- every later call fails the same way and teardown aborts the transport.
ftar_status_t first_contact(ftar_comm* c) {
  if (c->broken) {
    set_error("this communicator's first contact timed out earlier: it is unusable (destroy it)", __FILE__, __LINE__);
    return FTAR_ERR_TIMEOUT;
  }
  const char* e = getenv("FTAR_FIRST_CONTACT_TIMEOUT_S");
  const double limit = e && *e ? atof(e) : 600.0;
  auto run = [](ftar_comm* cc) {
    ftar_status_t st = agree_settings(cc);
    if (st == FTAR_SUCCESS) st = cc->tp->connect_peers(cc->rank);
    return st;
  };
  if (!c->tp->first_contact_blocks() || limit <= 0) return run(c);
  auto fc = std::make_shared<FirstContact>();
  c->contact = fc;
  c->contact_thread = std::thread([c, fc, run] {
    hip_ignore(hipSetDevice(c->device));
    const ftar_status_t st = run(c);
    std::lock_guard<std::mutex> g(fc->mu);
    fc->st = st;
    fc->err = st == FTAR_SUCCESS ? "" : last_error();
    fc->done = true;
    fc->cv.notify_all();
  });
  std::unique_lock<std::mutex> lk(fc->mu);
  if (!fc->cv.wait_for(lk, std::chrono::duration<double>(limit), [&] { return fc->done; })) {
    c->broken = true;
    set_error("first contact of the RCCL communicator (settings all-gather, p2p connections) not complete after " +
                  std::to_string(limit) + " s: a peer is missing or the transport is stuck; the communicator is "
                  "unusable (FTAR_FIRST_CONTACT_TIMEOUT_S)",
              __FILE__, __LINE__);
    return FTAR_ERR_TIMEOUT;
  }
  const ftar_status_t st = fc->st;
  const std::string err = fc->err;
  lk.unlock();
  c->contact_thread.join();
  if (st != FTAR_SUCCESS) set_error("first contact: " + err, __FILE__, __LINE__);
  return st;
}

// The topology of a call with topo == NULL, from the environment AT THIS CALL
// (get_stages, mpi_mod.hpp:1419-1486, re-run by every MPI_Allreduce_FT call,
// :1732).  FT_TOPO and FT_LONELY both unset (or FT_LONELY "0"): *is_auto, the
// cost model chooses (the reference exit(1)s here for P > 1).
// Anything else must parse for this communicator's size, or the call fails
// with FTAR_ERR_INVALID_TOPO before it enqueues anything (the reference:
// "invalid FT_TOPO" and exit(1), :1471-1475) -- on every rank alike, since
// every rank reads the same environment.
static ftar_status_t env_topology(ftar_comm* c, bool* is_auto, Topology* out) {
  const char* et = getenv("FT_TOPO");
  const char* el = getenv("FT_LONELY");
  const std::string st = et ? et : "", sl = el ? el : "";
  if (!c->env_seen || st != c->env_topo || sl != c->env_lonely) {
    c->env_seen = true;
    c->env_topo = st;
    c->env_lonely = sl;
    c->env_auto = st.empty() && (sl.empty() || sl == "0");
    c->env_status = FTAR_SUCCESS;
    if (!c->env_auto) {
      ftar_topo_t t;
      c->env_status = ftar_topo_parse(st.c_str(), sl.c_str(), c->nranks, &t);
      if (c->env_status == FTAR_SUCCESS) c->env_status = to_topology(&t, c->nranks, &c->env_t);
      if (c->env_status != FTAR_SUCCESS) c->env_status = FTAR_ERR_INVALID_TOPO;
    }
  }
  if (c->env_status != FTAR_SUCCESS) {
    set_error("invalid FT_TOPO '" + st + "' / FT_LONELY '" + sl + "' for " + std::to_string(c->nranks) + " ranks",
              __FILE__, __LINE__);
    return c->env_status;
  }
  *is_auto = c->env_auto;
  if (!c->env_auto) *out = c->env_t;
  return FTAR_SUCCESS;
}

// false: the communicator must not be freed (its first contact's helper thread may still be inside the
// transport after the abort; it is left behind with the memory it uses)
bool comm_teardown(ftar_comm* c) {
  hip_ignore(hipSetDevice(c->device));
  if (c->contact_thread.joinable()) {
    if (c->broken && c->tp) c->tp->abort();  // ncclCommAbort: the stuck first contact returns with an error
    bool done = false;
    {
      std::unique_lock<std::mutex> lk(c->contact->mu);
      done = c->contact->cv.wait_for(lk, std::chrono::seconds(c->broken ? 10 : 600), [&] { return c->contact->done; });
    }
    if (!done) {
      c->contact_thread.detach();
      return false;
    }
    c->contact_thread.join();
  }
  // A broken communicator's transport is aborted and its first-contact helper has returned: everything is
  // released as usual, only its streams are not waited for (nothing on them is waited for after an abort)
  if (!c->broken)
    for (hipStream_t st : {c->comm_s, c->red_s, c->h2d_s, c->d2h_s})
      if (st) hip_ignore(hipStreamSynchronize(st));
  if (c->tp) {
    c->tp->unmap_peers(&c->xpeers, c->rank);
    for (auto& r : c->regs) {
      c->tp->unmap_peers(&r.second.peers, c->rank);
      c->tp->rccl_deregister(r.second.rccl);
    }
    if (c->scratch_rccl) c->tp->rccl_deregister(c->scratch_rccl);
    c->scratch_rccl = nullptr;
  }
  c->regs.clear();
  if (c->xbuf) {
    forget_token(c->xbuf);
    hip_ignore(hipFree(c->xbuf));
  }
  c->tp.reset();
  for (hipStream_t t : c->dma_s) hip_ignore(hipStreamDestroy(t));
  for (hipEvent_t e : c->dma_ev) hip_ignore(hipEventDestroy(e));
  if (c->dma_fork) hip_ignore(hipEventDestroy(c->dma_fork));
  if (c->done_ev) hip_ignore(hipEventDestroy(c->done_ev));
  for (auto e : c->events) hip_ignore(hipEventDestroy(e));
  for (auto e : c->captured_events) hip_ignore(hipEventDestroy(e));
  for (auto e : c->tev) hip_ignore(hipEventDestroy(e));
  if (c->scratch) hip_ignore(hipFree(c->scratch));
  if (c->staging) hip_ignore(hipFree(c->staging));
  if (c->glog.host) hip_ignore(hipHostFree(c->glog.host));
  if (c->glog.dev) hip_ignore(hipFree(c->glog.dev));
  for (hipStream_t st : {c->comm_s, c->red_s, c->h2d_s, c->d2h_s})
    if (st) hip_ignore(hipStreamDestroy(st));
  return true;
}

namespace {

// The call's topology: the argument, or FT_TOPO/FT_LONELY read at this call; both unset: *is_auto (the
// execution model chooses), or under FTAR_COST_MODEL=reference the reference's own model's width list.
ftar_status_t call_topology(ftar_comm* c, const ftar_topo_t* topo, size_t bytes, Topology* t, bool* is_auto) {
  *is_auto = false;
  if (topo) return to_topology(topo, c->nranks, t);
  FTAR_RETURN_IF(env_topology(c, is_auto, t));
  const char* m = getenv("FTAR_COST_MODEL");
  if (*is_auto && m && !strcmp(m, "reference")) {
    ftar_topo_t ch;
    FTAR_RETURN_IF(ftar_topo_choose(c->nranks, bytes, &ch));
    FTAR_RETURN_IF(to_topology(&ch, c->nranks, t));
    *is_auto = false;
  }
  return FTAR_SUCCESS;
}

// What the call runs: the topology, form and piece the caller fixed, the rest from the execution model
// (cost_model.cpp), cached per communicator.  The same inputs on every rank give the same choice: the
// model's constants are compared across ranks at the first call (agree_settings).  Peer forms are
// candidates only for device buffers (captured or not: a capture takes the choice its warm-up call took),
// only at P > 1, and only once their rates are set.
ftar_status_t decide_exec(ftar_comm* c, Topology* t, bool topo_auto, size_t bytes, bool host, ExecChoice* out) {
  int flags = 0;
  if (topo_auto) flags |= FTAR_CHOOSE_TOPO;
  if (c->form == FTAR_FORM_AUTO && c->tp->async_p2p()) {
    flags |= FTAR_CHOOSE_FORM;
    // the same choice captured or not: a warm-up call of the shape sizes exactly what its capture uses
    if (!host && c->nranks > 1) flags |= FTAR_CHOOSE_PEER;
  }
  if (!c->chunk_bytes && !host) flags |= FTAR_CHOOSE_CHUNK;
  // a fixed mix of settings no form names is priced as the form of its reduce-scatter
  const int fixed_form = c->form >= FTAR_FORM_DIRECT ? c->form
                         : c->reduce_scatter == FTAR_RS_STAGES ? FTAR_FORM_STAGES : FTAR_FORM_DIRECT;
  const size_t fixed_chunk = host ? 0 : c->chunk_bytes;
  const std::string key = std::to_string(bytes) + "/" + std::to_string(flags) + "/" + t->key() + "/" +
                          std::to_string(fixed_form) + "/" + std::to_string(fixed_chunk) + "/" +
                          std::to_string(cost_generation());
  auto it = c->exec_cache.find(key);
  if (it == c->exec_cache.end()) {
    ExecChoice ch;
    ftar_status_t st = choose_exec(c->nranks, bytes, flags, *t, fixed_form, fixed_chunk, &ch);
    if (st != FTAR_SUCCESS) {  // nothing the model can price (e.g. P > FTAR_MAX_K one-round): as configured
      ch.topo = *t;
      ch.form = fixed_form;
      ch.chunk = fixed_chunk;
      ch.seconds = -1;
      if (flags & FTAR_CHOOSE_TOPO) {  // the topology the default data movement would take (ftar_topo_choose)
        ExecChoice d;
        if (choose_exec(c->nranks, bytes, FTAR_CHOOSE_TOPO | FTAR_CHOOSE_CHUNK, *t, FTAR_FORM_DIRECT, 0, &d) ==
            FTAR_SUCCESS) {
          ch.topo = d.topo;
        } else {  // the ring runs at any size
          ch.topo = Topology();
          ch.topo.ring = true;
          ch.topo.widths = {1};
        }
      }
    }
    if (c->exec_cache.size() > 256) c->exec_cache.clear();
    it = c->exec_cache.emplace(key, ch).first;
  }
  *out = it->second;
  *t = out->topo;
  return FTAR_SUCCESS;
}

// The call's cached plan; check_world once per (topology, count, form).
ftar_status_t resolve_plan(ftar_comm* c, const Topology& t, size_t count, const Form& form, const Plan** out) {
  const std::string key = t.key() + "/" + std::to_string(count) + "/ag" + std::to_string(form.allgather) + "/rs" +
                          std::to_string(form.reduce_scatter);
  auto it = c->plans.find(key);
  if (it == c->plans.end()) {
    auto p = std::make_shared<Plan>();
    FTAR_RETURN_IF(check_world(t, c->nranks, count, form));
    FTAR_RETURN_IF(build_plan(t, c->nranks, c->rank, count, p.get(), form));
    if (c->plans.size() > 64) c->plans.clear();
    it = c->plans.emplace(key, p).first;
  }
  if (it->second->max_k > FTAR_MAX_K) return FTAR_ERR_UNSUPPORTED;
  *out = it->second.get();
  return FTAR_SUCCESS;
}

// Grow-only device buffer; before freeing the old one, drain the streams whose
// earlier work may still touch it.
ftar_status_t ensure_buffer(void** buf, size_t* have, size_t need, std::initializer_list<hipStream_t> users) {
  if (need <= *have) return FTAR_SUCCESS;
  if (*buf) {
    for (hipStream_t st : users)
      if (st) FTAR_CHECK_HIP(hipStreamSynchronize(st));  // (a stream not created yet has nothing in flight)
    FTAR_CHECK_HIP(hipFree(*buf));
    *buf = nullptr;
    *have = 0;
  }
  FTAR_CHECK_ALLOC(hipMalloc(buf, need));
  *have = need;
  return FTAR_SUCCESS;
}

// Per-stage dependency facts of a plan: does it move / reduce / receive into
// scratch, the latest reducing stage before it (its data), and in the
// stage-major order the last reader of the scratch half it receives into.
struct StageFacts {
  std::vector<char> moves, reduces, to_scratch;
  std::vector<long> prev_red, war;
  explicit StageFacts(const Plan& plan) {
    const size_t nst = plan.stages.size();
    moves.assign(nst, 0);
    reduces.assign(nst, 0);
    to_scratch.assign(nst, 0);
    prev_red.assign(nst, -1);
    war.assign(nst, -1);
    long last = -1, owner[2] = {-1, -1};
    for (size_t s = 0; s < nst; ++s) {
      const Stage& st = plan.stages[s];
      moves[s] = !st.sends.empty() || !st.recvs.empty();
      reduces[s] = !st.reduces.empty();
      for (const Transfer& x : st.recvs) to_scratch[s] |= x.buf == BUF_SCRATCH;
      prev_red[s] = last;
      war[s] = to_scratch[s] ? owner[s % 2] : -1;
      if (reduces[s]) {
        last = (long)s;
        if (to_scratch[s]) owner[s % 2] = (long)s;
      }
    }
  }
};

// Skewed execution gives every stage its own scratch region: delta[s] moves a
// stage's scratch offsets from its alternating half to that region.  Returns
// the scratch elements needed.
size_t per_stage_scratch(const Plan& plan, std::vector<long>* delta) {
  const size_t nst = plan.stages.size();
  delta->assign(nst, 0);
  size_t base = 0;
  for (size_t s = 0; s < nst; ++s) {
    const size_t half_base = (s % 2) * plan.scratch_half;
    size_t used = 0;
    for (const Transfer& x : plan.stages[s].recvs)
      if (x.buf == BUF_SCRATCH) used = std::max(used, x.off - half_base + x.len);
    (*delta)[s] = (long)base - (long)half_base;
    base += used;
  }
  return base;
}

// Order of the (stage, piece) steps, identical on every rank.  Stage-major, or
// skewed: stage s+1 trails stage s by one piece.
std::vector<std::pair<size_t, size_t>> step_order(size_t nst, size_t nchunks, bool skew) {
  std::vector<std::pair<size_t, size_t>> order;
  order.reserve(nst * nchunks);
  if (!skew) {
    for (size_t s = 0; s < nst; ++s)
      for (size_t k = 0; k < nchunks; ++k) order.emplace_back(s, k);
  } else {
    for (size_t tt = 0; tt < nchunks + nst - 1; ++tt)
      for (size_t s = 0; s < nst && s <= tt; ++s)
        if (tt - s < nchunks) order.emplace_back(s, tt - s);
  }
  return order;
}

}  // namespace

ftar_status_t allreduce_locked(const void* sendbuf, void* recvbuf, size_t count, ftar_dtype_t dt, ftar_op_t op,
                               const ftar_topo_t* topo, ftar_comm* c, hipStream_t stream, const HostIO* host);

// One call on a communicator.  Calls share the communicator's scratch, staging
// and exchange buffers; the internal streams join the caller's stream at entry,
// so calls on ONE stream are ordered by it.  A call on another stream than the
// previous call's first waits for that call's completion marker (recorded on
// its stream after every internal stream joined it), so its transfers cannot
// overwrite scratch the previous call's reduces are still reading.
// Serial capture: a captured call issues everything on the caller's stream (FTAR_CAPTURE_SERIAL=1 / 0;
// default on when the loaded HIP runtime is older than 7.2).  torch 2.10 bundles HIP 7.0, whose
// hipStreamEndCapture dies (SIGSEGV, unbounded recursion) on the graph the forked comm/reduce streams and
// their per-piece cross waits leave, while 7.2 captures it; a chain in issue order keeps every
// dependency and gives up only the comm/reduce overlap inside the graph.
bool serial_capture() {
  static const bool on = [] {
    if (const char* e = getenv("FTAR_CAPTURE_SERIAL")) return *e != '0';
    int v = 0;
    return hipRuntimeGetVersion(&v) != hipSuccess || v < 70200000;  // major*1e7 + minor*1e5 + patch
  }();
  return on;
}

ftar_status_t allreduce(const void* sendbuf, void* recvbuf, size_t count, ftar_dtype_t dt, ftar_op_t op,
                        const ftar_topo_t* topo, ftar_comm* c, hipStream_t stream, const HostIO* host) {
  if (!c) return FTAR_ERR_INVALID_ARG;
  if (!dtype_op_supported(dt, op)) return FTAR_ERR_UNSUPPORTED;
  if (!recvbuf) {  // MPI allows null buffers with count 0 (e.g. an empty pinned tensor): nothing to do
    if (count) set_error("recvbuf is NULL", __FILE__, __LINE__);
    return count ? FTAR_ERR_INVALID_ARG : FTAR_SUCCESS;
  }
  std::lock_guard<std::mutex> g(c->mu);
  FTAR_CHECK_HIP(hipSetDevice(c->device));
  // under capture the graph's own dependencies order its replays: an event recorded outside the capture
  // is not waited on inside it, nor is the marker re-recorded by a captured call
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  FTAR_CHECK_HIP(hipStreamIsCapturing(stream, &cs));
  const bool capturing = cs != hipStreamCaptureStatusNone;
  if (capturing && !c->tp->async_p2p() && c->nranks > 1) {  // its barriers synchronise the host
    set_error("a host-bootstrapped communicator cannot run under stream capture (its barriers synchronise the host)",
              __FILE__, __LINE__);
    return FTAR_ERR_UNSUPPORTED;
  }
  if (!capturing && c->done_recorded && c->done_stream != stream)
    FTAR_CHECK_HIP(hipStreamWaitEvent(stream, c->done_ev, 0));
  c->capturing = capturing;
  // serial capture: every internal stream is the caller's for this call, so the captured graph is one
  // chain in issue order (every wait refers to an event recorded earlier in that order, so the chain keeps
  // every dependency; the comm/reduce overlap is given up inside the graph)
  const bool serial = capturing && (serial_capture() || c->tp->capture_serially());
  if (host) FTAR_RETURN_IF(ensure_host_streams(c));
  hipStream_t saved[4] = {c->comm_s, c->red_s, c->h2d_s, c->d2h_s};
  if (serial) c->comm_s = c->red_s = c->h2d_s = c->d2h_s = stream;
  c->serial = serial;
  const ftar_status_t st = allreduce_locked(sendbuf, recvbuf, count, dt, op, topo, c, stream, host);
  if (serial) c->comm_s = saved[0], c->red_s = saved[1], c->h2d_s = saved[2], c->d2h_s = saved[3];
  c->serial = false;
  c->capturing = false;
  if (st == FTAR_SUCCESS && !capturing) {
    FTAR_CHECK_HIP(hipEventRecord(c->done_ev, stream));
    c->done_stream = stream;
    c->done_recorded = true;
  }
  return st;
}

ftar_status_t allreduce_locked(const void* sendbuf, void* recvbuf, size_t count, ftar_dtype_t dt, ftar_op_t op,
                               const ftar_topo_t* topo, ftar_comm* c, hipStream_t stream, const HostIO* host) {
  const size_t esz = dtype_size(dt);
  if (sendbuf == recvbuf) sendbuf = nullptr;
  {  // the topology is checked first, as get_stages runs before the P <= 1 copy (mpi_mod.hpp:1732-1746)
    Topology t;
    bool is_auto = false;
    FTAR_RETURN_IF(topo ? to_topology(topo, c->nranks, &t) : env_topology(c, &is_auto, &t));
  }
  if (c->broken) return first_contact(c);  // reports why
  if (!c->settings_agreed && !c->capturing) {  // an RCCL communicator's first call (see comm_setup); a
    FTAR_RETURN_IF(first_contact(c));          // 1-rank one too, which exercises the same all-gather
    c->settings_agreed = true;
  }
  if (c->nranks == 1) {  // mpi_mod.hpp:1739-1746
    if (sendbuf && count && host)
      FTAR_CHECK_HIP(hipMemcpyAsync(recvbuf, sendbuf, count * esz, hipMemcpyHostToHost, stream));
    if (sendbuf && count && !host) return launch_copy(sendbuf, recvbuf, count * esz, stream);
    return FTAR_SUCCESS;
  }
  if (count == 0) return FTAR_SUCCESS;

  Topology topology;
  bool topo_auto = false;
  FTAR_RETURN_IF(call_topology(c, topo, count * esz, &topology, &topo_auto));
  ExecChoice ex;
  FTAR_RETURN_IF(decide_exec(c, &topology, topo_auto, count * esz, host != nullptr, &ex));
  Form form;
  form.allgather = c->allgather;
  form.reduce_scatter = c->reduce_scatter;
  int peer_mode = c->peer_direct;
  if (c->form == FTAR_FORM_AUTO && c->tp->async_p2p())
    form_settings(ex.form, &form.allgather, &form.reduce_scatter, &peer_mode);
  if (host && form.allgather == FTAR_AG_COLLECTIVE) form.allgather = FTAR_AG_DIRECT;  // D2H needs pieces
  const Plan* planp = nullptr;
  FTAR_RETURN_IF(resolve_plan(c, topology, count, form, &planp));
  const Plan& plan = *planp;
  // what runs (ftar_comm_last_exec): the model's or the settings' form, unless the plan or the buffers send
  // the call down another path below (host buffers on a p2p transport, a plan no peer kernel runs, the
  // collective all-gather a ring or host buffers replace)
  const bool peer_path = peer_mode && peer_eligible(plan) && (!host || !c->tp->async_p2p());
  int ran = ex.form;
  if (peer_path) ran = peer_mode == FTAR_PEER_READ ? FTAR_FORM_PEER_READ : FTAR_FORM_PEER_WRITE;
  else if (form.reduce_scatter == FTAR_RS_STAGES) ran = plan.allgather == FTAR_AG_STAGES ? FTAR_FORM_STAGES : -2;
  else ran = plan.allgather == FTAR_AG_DIRECT ? FTAR_FORM_DIRECT
             : plan.allgather == FTAR_AG_COLLECTIVE ? FTAR_FORM_COLLECTIVE : -2;
  from_topology(topology, &c->last_exec.topo);
  c->last_exec.form = ran;
  c->last_exec.chunk_bytes = peer_path ? 0 : ex.chunk;  // the host paths below put the piece they run
  c->last_exec.seconds = ex.seconds;
  c->last_exec.tied = ex.tied;
  c->last_exec.tie_broken_by = ex.tie_broken_by;
  const size_t nst = plan.stages.size();
  if (!c->tp->async_p2p()) {
    // A host-bootstrapped communicator's paths differ in their host barriers (peer read: 3, write: 3,
    // host buffers pipelined: m + 2, whole bucket: 3), so every rank must take the same one with the same
    // pieces: the settings that choose it are compared first, and a mismatch fails the call on every rank
    //  instead of pairing barriers of different phases.
    const uint64_t cfg[6] = {(uint64_t)peer_mode, (uint64_t)c->allgather, (uint64_t)c->reduce_scatter,
                             (uint64_t)(host != nullptr), host ? (uint64_t)c->host_peer_pipeline : 0,
                             host ? (uint64_t)host_peer_piece(c, plan.split, esz) : 0};
    bool same = true;
    FTAR_RETURN_IF(c->tp->agree(cfg, sizeof cfg, &same));
    if (!same) {
      set_error("ranks disagree on the peer form, all-gather/reduce-scatter form, FTAR_HOST_PEER_PIPELINE or the "
                "host piece size (FTAR_HOST_CHUNK_BYTES): set them alike on every rank",
                __FILE__, __LINE__);
      return FTAR_ERR_INVALID_ARG;
    }
  }
  if (!host && peer_mode && peer_eligible(plan)) {
    FTAR_RETURN_IF(grow_events(c, 5));
    return peer_allreduce(sendbuf, recvbuf, count, dt, op, plan, c, stream, peer_mode);
  }
  if (host && peer_mode == FTAR_PEER_READ && !c->tp->async_p2p() && peer_eligible(plan) &&
      c->host_peer_pipeline && host_peer_piece(c, plan.split, esz) < plan.split) {
    // host buffers on a transport without p2p (a communicator bootstrapped over MPI with no RCCL,
    // ftar_comm_init_host): the read form piece by piece, H2D / exchange / D2H overlapped.  A bucket
    // of one piece per block gains nothing from it and takes the whole-bucket path below, whose one
    // copy each way beats one per block (C1 through the MPI harness: 0.453 vs 0.487 ms)
    FTAR_RETURN_IF(grow_events(c, 5));
    c->last_exec.chunk_bytes = host_peer_piece(c, plan.split, esz) * esz;
    return peer_allreduce_host(*host, count, dt, op, plan, c, stream);
  }
  if (host && peer_mode && !c->tp->async_p2p() && peer_eligible(plan)) {
    // the write form (or FTAR_HOST_PEER_PIPELINE=0): the whole bucket in, the peer exchange in HBM,
    // the whole bucket out -- same plan, same bits, not pipelined (transports with stream-ordered
    // p2p keep using the pipelined p2p path below for host buffers even in peer-direct mode)
    const size_t bytes = count * esz;
    if (bytes > c->staging_bytes) FTAR_RETURN_IF(refuse_growth_under_capture(c, "the staging buffer"));
    FTAR_RETURN_IF(ensure_buffer(&c->staging, &c->staging_bytes, bytes, {c->h2d_s, c->comm_s, c->red_s, c->d2h_s}));
    FTAR_CHECK_HIP(hipMemcpyAsync(c->staging, host->src, bytes, hipMemcpyHostToDevice, stream));
    FTAR_RETURN_IF(grow_events(c, 5));
    FTAR_RETURN_IF(peer_allreduce(nullptr, c->staging, count, dt, op, plan, c, stream, peer_mode));
    FTAR_CHECK_HIP(hipMemcpyAsync(host->dst, c->staging, bytes, hipMemcpyDeviceToHost, stream));
    return FTAR_SUCCESS;
  }

  if (!c->tp->async_p2p()) {  // a transport without p2p (ftar_comm_init_host): refused before anything moves
    set_error("this communicator has no point-to-point transfers: one-round plans in the peer-direct forms only "
              "(ftar_comm_set_peer_direct; staged forms and lonely ranks need RCCL)",
              __FILE__, __LINE__);
    return FTAR_ERR_UNSUPPORTED;
  }

  // Host mode: the buffers are in host memory and move through a device
  // staging buffer, piece by piece, so H2D (PCIe in), the exchange, and D2H
  // (PCIe out) run at the same time.  Every src/dst transfer and reduce of a
  // plan covers whole blocks from their start (tests/test_plan.py), so piece
  // k of every stage touches exactly piece k of each block: the same bytes,
  // the same partition, the same bits as the device path.
  // the piece: fixed, or the model's (0 = whole blocks)
  size_t chunk_bytes = c->chunk_bytes ? c->chunk_bytes : ex.chunk ? ex.chunk : plan.split * esz;
  if (host) {
    chunk_bytes = c->host_chunk_bytes ? c->host_chunk_bytes : auto_host_chunk(plan.split * esz);
    c->last_exec.chunk_bytes = std::max<size_t>(64, (chunk_bytes / esz) & ~size_t(63)) * esz;  // the piece run
    if (count * esz > c->staging_bytes) FTAR_RETURN_IF(refuse_growth_under_capture(c, "the staging buffer"));
    FTAR_RETURN_IF(ensure_buffer(&c->staging, &c->staging_bytes, count * esz, {c->h2d_s, c->comm_s, c->red_s, c->d2h_s}));
    sendbuf = nullptr;
    recvbuf = c->staging;
  }
  const size_t chunk = std::max<size_t>(64, (chunk_bytes / esz) & ~size_t(63));
  const size_t nchunks = std::max<size_t>(1, (plan.split + chunk - 1) / chunk);
  const StageFacts f(plan);
  const std::vector<char>& moves = f.moves;
  const std::vector<char>& reduces = f.reduces;
  const std::vector<long>& prev_red = f.prev_red;
  const std::vector<long>& war = f.war;
  // Device: stage-major.  Host: skewed, so the all-gather of piece k (and its
  // D2H) runs while later pieces are still coming in over PCIe; skewed steps
  // of stages two apart may overlap in time, so every stage gets its own
  // scratch region instead of alternating halves.
  const bool skew = host != nullptr;
  std::vector<long> delta(nst, 0);
  const size_t scratch_elems = skew ? per_stage_scratch(plan, &delta) : 2 * plan.scratch_half;
  if (scratch_elems * esz > c->scratch_bytes) {
    FTAR_RETURN_IF(refuse_growth_under_capture(c, "the scratch buffer"));
    if (c->scratch_rccl) {  // the old scratch is about to be freed: drop its RCCL registration first
      FTAR_CHECK_HIP(hipStreamSynchronize(c->comm_s));
      FTAR_CHECK_HIP(hipStreamSynchronize(c->red_s));
      c->tp->rccl_deregister(c->scratch_rccl);
      c->scratch_rccl = nullptr;
    }
  }
  FTAR_RETURN_IF(ensure_buffer(&c->scratch, &c->scratch_bytes, scratch_elems * esz, {c->comm_s, c->red_s}));
  if (c->rccl_reg && !c->scratch_rccl && c->scratch && !c->capturing)
    c->scratch_rccl = c->tp->rccl_register(c->scratch, c->scratch_bytes);
  const std::vector<std::pair<size_t, size_t>> order = step_order(nst, nchunks, skew);

  FTAR_RETURN_IF(grow_events(c, 2 * nst * nchunks + 2 * nchunks + 5));
  hipEvent_t* ev = c->events.data();
  auto ev_x = [&](size_t s, size_t k) { return ev[5 + (s * nchunks + k) * 2]; };
  auto ev_r = [&](size_t s, size_t k) { return ev[5 + (s * nchunks + k) * 2 + 1]; };
  auto ev_h = [&](size_t k) { return ev[5 + 2 * nst * nchunks + 2 * k]; };
  auto ev_d = [&](size_t k) { return ev[5 + 2 * nst * nchunks + 2 * k + 1]; };

  char* bufs[3] = {static_cast<char*>(const_cast<void*>(sendbuf ? sendbuf : recvbuf)), static_cast<char*>(recvbuf),
                   static_cast<char*>(c->scratch)};
  Transport* tp = c->tp.get();
  const size_t P = (size_t)c->nranks, split = plan.split;
  // piece k of every block: [b*split + k*chunk, ...) clipped to the block and to count
  auto for_piece = [&](size_t k, auto&& fn) -> ftar_status_t {
    for (size_t b = 0; b < P; ++b) {
      const size_t lo = b * split + k * chunk, end = std::min(count, (b + 1) * split);
      if (lo < end) FTAR_RETURN_IF(fn(lo, std::min(chunk, end - lo)));
    }
    return FTAR_SUCCESS;
  };

  FTAR_CHECK_HIP(hipEventRecord(ev[0], stream));
  FTAR_CHECK_HIP(hipStreamWaitEvent(c->comm_s, ev[0], 0));
  FTAR_CHECK_HIP(hipStreamWaitEvent(c->red_s, ev[0], 0));
  c->nmarks = 0;
  FTAR_RETURN_IF(mark(c, "start", c->comm_s));
  // Host mode: the pieces go in, in order, on their own stream, issued kHostLookahead pieces ahead of the
  // steps that read them rather than all up front.  The copy stream then runs ahead of the exchange by
  // that many pieces either way, and a stream that shares its hardware queue with it (8 streams of two
  // in-process ranks on HIP's 4 queues, or a caller's own streams) waits behind those few pieces, not
  // behind the whole bucket: with every piece issued first, two ranks on one GPU started the exchange only
  // once the last piece was in, and H2D and D2H never overlapped (profiles/r05/host_local/).
  size_t h2d_issued = 0;
  auto issue_h2d = [&](size_t upto) -> ftar_status_t {  // pieces [h2d_issued, upto] of every block
    for (; h2d_issued <= upto && h2d_issued < nchunks; ++h2d_issued) {
      const size_t k = h2d_issued;
      FTAR_RETURN_IF(for_piece(k, [&](size_t lo, size_t n) -> ftar_status_t {
        FTAR_CHECK_HIP(hipMemcpyAsync(bufs[BUF_DST] + lo * esz, host->src + lo * esz, n * esz,
                                      hipMemcpyHostToDevice, c->h2d_s));
        return FTAR_SUCCESS;
      }));
      FTAR_CHECK_HIP(hipEventRecord(ev_h(k), c->h2d_s));
    }
    return FTAR_SUCCESS;
  };
  if (host) {
    FTAR_CHECK_HIP(hipStreamWaitEvent(c->h2d_s, ev[0], 0));
    FTAR_CHECK_HIP(hipStreamWaitEvent(c->d2h_s, ev[0], 0));
    FTAR_RETURN_IF(issue_h2d(kHostLookahead));
  }
  std::vector<char> comm_has_input(host ? nchunks : 0), red_has_input(host ? nchunks : 0);
  std::vector<const void*> srcs;
  auto sbuf = [&](int buf, size_t off, size_t s) -> char* {
    return bufs[buf] + (buf == BUF_SCRATCH ? (size_t)((long)off + delta[s]) : off) * esz;
  };
  for (const auto& step : order) {
    const size_t s = step.first, k = step.second, lo = k * chunk;
    const Stage& st = plan.stages[s];
    if (host) FTAR_RETURN_IF(issue_h2d(k + kHostLookahead));
    if (moves[s]) {
      if (host && !comm_has_input[k]) {
        FTAR_CHECK_HIP(hipStreamWaitEvent(c->comm_s, ev_h(k), 0));
        comm_has_input[k] = 1;
      }
      // WAR on the scratch half this stage receives into (stage-major only):
      // every reduce that read it (stage s-2, or earlier when stages in between
      // were empty) must be done.  When stage s-1 reduced, its piece-0 event
      // already implies this (the reduce stream runs in order), so the wait is
      // free; it matters when s-1 was empty.
      if (!skew && k == 0 && war[s] >= 0)
        FTAR_CHECK_HIP(hipStreamWaitEvent(c->comm_s, ev_r((size_t)war[s], nchunks - 1), 0));
      if (prev_red[s] >= 0) FTAR_CHECK_HIP(hipStreamWaitEvent(c->comm_s, ev_r((size_t)prev_red[s], k), 0));
      FTAR_RETURN_IF(tp->group_start());
      for (const Transfer& x : st.sends)
        if (x.len > lo)
          FTAR_RETURN_IF(tp->send(sbuf(x.buf, x.off + lo, s), std::min(chunk, x.len - lo) * esz, x.peer, c->comm_s));
      for (const Transfer& x : st.recvs)
        if (x.len > lo)
          FTAR_RETURN_IF(tp->recv(sbuf(x.buf, x.off + lo, s), std::min(chunk, x.len - lo) * esz, x.peer, c->comm_s));
      FTAR_RETURN_IF(tp->group_end());
    }
    if (reduces[s]) {
      FTAR_CHECK_HIP(hipEventRecord(ev_x(s, k), c->comm_s));
      FTAR_CHECK_HIP(hipStreamWaitEvent(c->red_s, ev_x(s, k), 0));
      if (host && !red_has_input[k]) {
        FTAR_CHECK_HIP(hipStreamWaitEvent(c->red_s, ev_h(k), 0));
        red_has_input[k] = 1;
      }
      for (const ReduceItem& r : st.reduces) {
        if (r.len <= lo) continue;
        srcs.clear();
        for (const Operand& o : r.srcs) srcs.push_back(sbuf(o.buf, o.off + lo, s));
        FTAR_RETURN_IF(launch_reduce(srcs.data(), (int)srcs.size(), bufs[BUF_DST] + (r.off + lo) * esz,
                                     std::min(chunk, r.len - lo), dt, op, c->red_s, r.round_each, r.shape.data(),
                                     (int)r.shape.size()));
      }
      FTAR_CHECK_HIP(hipEventRecord(ev_r(s, k), c->red_s));
    }
    if (c->phase_timing && !skew && k == nchunks - 1) {  // stage-major: the stage's last piece
      if (moves[s]) FTAR_RETURN_IF(mark(c, "stage " + std::to_string(s) + " moved", c->comm_s));
      if (reduces[s]) FTAR_RETURN_IF(mark(c, "stage " + std::to_string(s) + " reduced", c->red_s));
    }
    if (host && s == nst - 1) {  // piece k is final everywhere: out over PCIe while later pieces come in
      FTAR_CHECK_HIP(hipEventRecord(ev_d(k), reduces[s] ? c->red_s : c->comm_s));
      if (reduces[s]) FTAR_CHECK_HIP(hipStreamWaitEvent(c->d2h_s, ev_x(s, k), 0));
      else if (prev_red[s] >= 0)  // a rank idle in the last stage: its block's final fold
        FTAR_CHECK_HIP(hipStreamWaitEvent(c->d2h_s, ev_r((size_t)prev_red[s], k), 0));
      FTAR_CHECK_HIP(hipStreamWaitEvent(c->d2h_s, ev_d(k), 0));
      FTAR_RETURN_IF(for_piece(k, [&](size_t lo2, size_t n) -> ftar_status_t {
        FTAR_CHECK_HIP(hipMemcpyAsync(host->dst + lo2 * esz, bufs[BUF_DST] + lo2 * esz, n * esz,
                                      hipMemcpyDeviceToHost, c->d2h_s));
        return FTAR_SUCCESS;
      }));
    }
  }
  if (host) FTAR_RETURN_IF(issue_h2d(nchunks - 1));  // (every piece is read by a step; kept for safety)
  if (plan.allgather == FTAR_AG_COLLECTIVE) {  // the whole all-gather phase as one collective, in place
    const long last_red = nst ? (reduces[nst - 1] ? (long)nst - 1 : prev_red[nst - 1]) : -1;
    if (last_red >= 0) FTAR_CHECK_HIP(hipStreamWaitEvent(c->comm_s, ev_r((size_t)last_red, nchunks - 1), 0));
    FTAR_RETURN_IF(tp->allgather(bufs[BUF_DST] + (size_t)c->rank * plan.split * esz, bufs[BUF_DST], plan.split * esz,
                                 c->rank, c->nranks, c->comm_s));
  }
  if (plan.allgather == FTAR_AG_COLLECTIVE) FTAR_RETURN_IF(mark(c, "collective all-gather", c->comm_s));
  FTAR_RETURN_IF(tp->before_join());
  FTAR_CHECK_HIP(hipEventRecord(ev[1], c->comm_s));
  FTAR_CHECK_HIP(hipEventRecord(ev[2], c->red_s));
  FTAR_CHECK_HIP(hipStreamWaitEvent(stream, ev[1], 0));
  FTAR_CHECK_HIP(hipStreamWaitEvent(stream, ev[2], 0));
  if (host) {
    FTAR_CHECK_HIP(hipEventRecord(ev[3], c->h2d_s));
    FTAR_CHECK_HIP(hipEventRecord(ev[4], c->d2h_s));
    FTAR_CHECK_HIP(hipStreamWaitEvent(stream, ev[3], 0));
    FTAR_CHECK_HIP(hipStreamWaitEvent(stream, ev[4], 0));
  }
  return FTAR_SUCCESS;
}

}  // namespace ftar

// ============================================================================
// C ABI: communicators and AllReduce
// ============================================================================
