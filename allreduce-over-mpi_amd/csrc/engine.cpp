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

#include "ftar_internal.h"

using ftar::hip_ignore;

// The outcome of a communicator's first contact, shared with the helper thread that runs it.
struct FirstContact {
  std::mutex mu;
  std::condition_variable cv;
  bool done = false;
  ftar_status_t st = FTAR_SUCCESS;
  std::string err;
};

struct ftar_comm {
  int rank = 0, nranks = 1, device = 0;
  std::unique_ptr<ftar::Transport> tp;
  hipStream_t comm_s = nullptr, red_s = nullptr;
  hipStream_t h2d_s = nullptr, d2h_s = nullptr;  // host mode (ftar_allreduce_host), created at its first call
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  void* staging = nullptr;  // host mode: the device copy of the bucket, grow-only
  size_t staging_bytes = 0;
  size_t chunk_bytes = 0;  // the fixed pipeline piece; 0 = the execution model's per call (chunk_auto)
  size_t host_chunk_bytes = 0;
  // FTAR_FORM_AUTO: the execution model picks the form per call (cost_model.cpp); otherwise the form the
  // explicit settings below (allgather, reduce_scatter, peer_direct) describe, or -2 for a mix
  int form = FTAR_FORM_AUTO;
  // choices of the model, cached per (bytes, flags, fixed topology/form/piece, constants' generation)
  std::map<std::string, ftar::ExecChoice> exec_cache;
  ftar_exec_t last_exec{};
  int peer_direct = 0;             // FTAR_PEER_DIRECT / ftar_comm_set_peer_direct: 0 off, 1 read, 2 write
  // peer-form tuning (ftar_debug_set_peer_tuning; bench.py sweeps both on a
  // real node): nontemporal copies, LDS-staged fold (false: register kernel)
  bool peer_nt = true, peer_lds = true;
  // peer_dma: the xGMI copies of the peer forms (gather, scatter, push) by the DMA engines, one
  // hipMemcpyAsync per peer on its own stream forked from and joined back into comm_s
  bool peer_dma = false;
  // workgroups per segment of the cross-GPU copy kernels (gather, scatter, push); 0 = as many as the
  // segment fills (ftar_debug_set_peer_wg_cap; bench.py tries the xGMI probe's best cap when it beats that)
  size_t peer_wg_cap = 0;
  std::vector<hipStream_t> dma_s;
  std::vector<hipEvent_t> dma_ev;
  hipEvent_t dma_fork = nullptr;
  void* xbuf = nullptr;            // peer-direct exchange buffer (IPC-exported), grow-only
  size_t xbuf_bytes = 0;
  std::vector<char*> xpeers;       // every rank's exchange buffer, mapped here
  // registered user buffers (ftar_comm_register): id -> my range + every rank's
  // matching pointer, mapped here; the peer forms read/write them in place
  struct Reg {
    char* ptr;
    size_t bytes;
    std::vector<char*> peers;
    void* rccl = nullptr;  // ncclCommRegister handle (RCCL communicators), or nullptr
  };
  std::map<int, Reg> regs;
  int next_reg = 1;
  int allgather = FTAR_AG_DIRECT;
  int reduce_scatter = FTAR_RS_DIRECT;
  bool settings_agreed = false;  // agree_settings ran (engine.cpp comm_setup / the first call)
  // the first contact (first_contact) did not finish within its deadline: every call fails with
  // FTAR_ERR_TIMEOUT, and teardown aborts the transport instead of draining it
  bool broken = false;
  std::thread contact_thread;  // the first contact's helper (joined, or left behind on a broken communicator)
  std::shared_ptr<struct FirstContact> contact;
  // the scratch buffer registered with RCCL (ncclCommRegister), so p2p receives may land in it without
  // RCCL's staging copies (FTAR_RCCL_REGISTER=1 / ftar_debug_set_rccl_register; bench.py sweeps it)
  bool rccl_reg = false;
  void* scratch_rccl = nullptr;
  // FT_TOPO / FT_LONELY are read on every call with topo == NULL, as the
  // reference's get_stages is (mpi_mod.hpp:1732); the last strings seen and
  // what they parsed to are kept, so an unchanged environment costs two getenv
  bool env_seen = false;
  std::string env_topo, env_lonely;  // the strings last parsed ("" = unset)
  ftar_status_t env_status = FTAR_SUCCESS;
  bool env_auto = true;              // both unset: the cost model's choice per call
  ftar::Topology env_t;
  std::map<std::string, std::shared_ptr<ftar::Plan>> plans;
  std::vector<hipEvent_t> events;
  // phase timing (diagnostic, ftar_comm_set_phase_timing): timing events
  // recorded at the phase boundaries of the last call, in issue order
  bool phase_timing = false;
  std::vector<hipEvent_t> tev;
  std::vector<std::string> tnames;
  size_t nmarks = 0;
  // completion marker of the previous call, recorded on that call's stream after it joined every internal
  // stream: a call on a different stream waits for it (scratch, staging and exchange buffers are shared)
  hipEvent_t done_ev = nullptr;
  hipStream_t done_stream = nullptr;
  bool done_recorded = false;
  int reduce_cus = 0;      // CUs the reduce stream may use (0 = all; ftar_comm_set_reduce_cus)
  // host buffers on a host-bootstrapped communicator in the read form: piece-pipelined
  // (peer_allreduce_host); FTAR_HOST_PEER_PIPELINE=0 takes the whole-bucket path instead (A/B)
  bool host_peer_pipeline = true;
  bool capturing = false;  // the current call's stream is being captured: no allocation, no host sync
  bool serial = false;     // ... and every internal stream is the caller's (serial_capture)
  // events handed to captured calls: each captured call records a fresh set
  // (an event is never re-recorded inside one capture), kept until teardown
  std::vector<hipEvent_t> captured_events;
  std::mutex mu;
};

namespace ftar {

namespace {
// Host mode pieces (0 = auto): 16 MiB per block, at least split/64 (bounds the
// number of copies for huge buckets).  4 MiB device->host copies run at only
// ~33 GB/s; larger pieces lengthen the pipeline's fill and drain (one piece of
// every block each).  16 MiB was the best or near-best size in every sweep
// (profiles/r01/host/): 8 pieces per block at P = 8 x 1 GiB.
constexpr size_t kDefaultHostChunkBytes = 0;
constexpr size_t kMaxHostPeerPieces = 1024;  // peer_allreduce_host: pieces per call (a host barrier each)
size_t auto_host_chunk(size_t split_bytes) { return std::max<size_t>(16u << 20, split_bytes / 64); }

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
                  "stream on a hardware queue of its own, and over RCCL it stalled ranks (DESIGN §4); "
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
}  // namespace

// the host-buffer path's copy streams, created at the first host-buffer call (see comm_setup_local)
ftar_status_t ensure_host_streams(ftar_comm* c) {
  if (!c->h2d_s) FTAR_CHECK_HIP(hipStreamCreateWithFlags(&c->h2d_s, hipStreamNonBlocking));
  if (!c->d2h_s) FTAR_CHECK_HIP(hipStreamCreateWithFlags(&c->d2h_s, hipStreamNonBlocking));
  return FTAR_SUCCESS;
}

ftar_status_t agree_settings(ftar_comm* c, bool failed = false);

namespace {
// the local part of a communicator's bring-up: streams, events, settings from the environment
ftar_status_t comm_setup_local(ftar_comm* c) {
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
  for (hipStream_t st : {c->comm_s, c->red_s, c->h2d_s, c->d2h_s})
    if (st) hip_ignore(hipStreamDestroy(st));
  return true;
}

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

namespace {
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
template <class Where>
ftar_status_t peer_fold(const ReduceItem& r, const Plan& plan, ftar_dtype_t dt, ftar_op_t op, void* dst,
                        hipStream_t s, bool lds, Where where, size_t lo = 0, size_t len = SIZE_MAX) {
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
}  // namespace

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

namespace {
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
}  // namespace

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

// Host mode: sendbuf/recvbuf of the call are host memory (pinned for overlap).
struct HostIO {
  const char* src;
  char* dst;
};

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

// Host buffers on a communicator without point-to-point transfers (ftar_comm_init_host: the MPI
// drop-in's `ipc` transport), the read form piece by piece, as the p2p host path pipelines its
// stages.  Piece k is elements [k*chunk, (k+1)*chunk) of every block.
//   * every piece goes H2D straight into the exchange buffer X on its own stream, all issued up
//     front, so the copy engines run ahead (no staging buffer, no copy-in pass);
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
  // Every rank goes through all m + 2 barriers whatever fails locally: `st` keeps this rank's first
  // failure, the work after it is skipped, and each barrier tells every rank whether any rank failed,
  // so all of them leave the call at the same barrier instead of some waiting in the next.
  ftar_status_t st = grow_events(c, 5 + 2 * m);
  auto work = [&](auto&& fn) {
    if (st == FTAR_SUCCESS) st = fn();
  };
  // a failed call leaves only after its copies stopped touching the caller's host buffers: H2D reads of
  // io.src and D2H writes of io.dst may still be in flight on their streams
  auto leave = [&]() -> ftar_status_t {
    for (hipStream_t s : {c->h2d_s, c->d2h_s, c->comm_s})
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
  work([&]() -> ftar_status_t {
    ev = c->events.data();
    FTAR_CHECK_HIP(hipEventRecord(ev[0], stream));
    for (hipStream_t s : {c->comm_s, c->h2d_s, c->d2h_s}) FTAR_CHECK_HIP(hipStreamWaitEvent(s, ev[0], 0));
    c->nmarks = 0;
    FTAR_RETURN_IF(mark(c, "start", c->comm_s));
    for (size_t k = 0; k < m; ++k) {
      FTAR_RETURN_IF(for_piece(k, [&](size_t lo, size_t n) -> ftar_status_t {
        FTAR_CHECK_HIP(hipMemcpyAsync(X + lo * esz, io.src + lo * esz, n * esz, hipMemcpyHostToDevice, c->h2d_s));
        return FTAR_SUCCESS;
      }));
      FTAR_CHECK_HIP(hipEventRecord(ev_h(k), c->h2d_s));
    }
    FTAR_CHECK_HIP(hipStreamWaitEvent(c->comm_s, ev_h(0), 0));
    return FTAR_SUCCESS;
  });
  if (!sync()) return leave();  // piece 0 is in everywhere
  work([&] { return mark(c, "piece 0 in", c->comm_s); });
  std::vector<Segment> segs;
  for (size_t k = 0; k < m; ++k) {
    const size_t lo = k * chunk;
    work([&]() -> ftar_status_t {
      for (const ReduceItem& r : rs.reduces)
        FTAR_RETURN_IF(peer_fold(
            r, plan, dt, op, X + (r.off + lo) * esz, c->comm_s, c->peer_lds,
            [&](int q, size_t off) -> const void* { return (q < 0 ? X : Xq[q]) + off * esz; }, lo, chunk));
      if (k + 1 < m) FTAR_CHECK_HIP(hipStreamWaitEvent(c->comm_s, ev_h(k + 1), 0));
      return FTAR_SUCCESS;
    });
    if (!sync()) return leave();  // piece k folded everywhere (and piece k+1 in)
    work([&]() -> ftar_status_t {
      segs.clear();
      for (const Transfer& x : ag.recvs)
        if (x.len > lo)
          segs.push_back(
              {Xq[x.peer] + (x.off + lo) * esz, X + (x.off + lo) * esz, std::min(chunk, x.len - lo) * esz});
      if (!segs.empty()) FTAR_RETURN_IF(peer_copy(c, segs));
      FTAR_CHECK_HIP(hipEventRecord(ev_g(k), c->comm_s));
      FTAR_CHECK_HIP(hipStreamWaitEvent(c->d2h_s, ev_g(k), 0));
      return for_piece(k, [&](size_t lo2, size_t n) -> ftar_status_t {
        FTAR_CHECK_HIP(
            hipMemcpyAsync(io.dst + lo2 * esz, X + lo2 * esz, n * esz, hipMemcpyDeviceToHost, c->d2h_s));
        return FTAR_SUCCESS;
      });
    });
  }
  work([&] { return mark(c, "pieces folded and gathered", c->comm_s); });
  if (!sync()) return leave();  // no peer reads my X after the call
  if (st != FTAR_SUCCESS) return leave();
  FTAR_RETURN_IF(mark(c, "barrier", c->comm_s));
  FTAR_RETURN_IF(tp->before_join());
  FTAR_CHECK_HIP(hipEventRecord(ev[1], c->comm_s));
  FTAR_CHECK_HIP(hipEventRecord(ev[2], c->d2h_s));
  FTAR_CHECK_HIP(hipEventRecord(ev[3], c->h2d_s));
  for (int i = 1; i <= 3; ++i) FTAR_CHECK_HIP(hipStreamWaitEvent(stream, ev[i], 0));
  return FTAR_SUCCESS;
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
                        const ftar_topo_t* topo, ftar_comm* c, hipStream_t stream, const HostIO* host = nullptr) {
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
  if (host) {  // all pieces in, in order, on their own stream (the DMA engines run ahead)
    FTAR_CHECK_HIP(hipStreamWaitEvent(c->h2d_s, ev[0], 0));
    FTAR_CHECK_HIP(hipStreamWaitEvent(c->d2h_s, ev[0], 0));
    for (size_t k = 0; k < nchunks; ++k) {
      FTAR_RETURN_IF(for_piece(k, [&](size_t lo, size_t n) -> ftar_status_t {
        FTAR_CHECK_HIP(hipMemcpyAsync(bufs[BUF_DST] + lo * esz, host->src + lo * esz, n * esz,
                                      hipMemcpyHostToDevice, c->h2d_s));
        return FTAR_SUCCESS;
      }));
      FTAR_CHECK_HIP(hipEventRecord(ev_h(k), c->h2d_s));
    }
  }
  std::vector<char> comm_has_input(host ? nchunks : 0), red_has_input(host ? nchunks : 0);
  std::vector<const void*> srcs;
  auto sbuf = [&](int buf, size_t off, size_t s) -> char* {
    return bufs[buf] + (buf == BUF_SCRATCH ? (size_t)((long)off + delta[s]) : off) * esz;
  };
  for (const auto& step : order) {
    const size_t s = step.first, k = step.second, lo = k * chunk;
    const Stage& st = plan.stages[s];
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
  *mode = static_cast<ftar_reduce_scatter_t>(comm->reduce_scatter);
  return FTAR_SUCCESS;
}

ftar_status_t ftar_comm_get_allgather(ftar_comm_t comm, ftar_allgather_t* mode) {
  if (!comm || !mode) return FTAR_ERR_INVALID_ARG;
  *mode = static_cast<ftar_allgather_t>(comm->allgather);
  return FTAR_SUCCESS;
}

ftar_status_t ftar_comm_get_chunk_bytes(ftar_comm_t comm, size_t* bytes) {
  if (!comm || !bytes) return FTAR_ERR_INVALID_ARG;
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

ftar_status_t ftar_comm_set_reduce_cus(ftar_comm_t comm, int cus) {
  if (!comm) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(comm->mu);
  FTAR_CHECK_HIP(hipSetDevice(comm->device));
  return ftar::set_reduce_cus(comm, cus);
}

ftar_status_t ftar_comm_get_reduce_cus(ftar_comm_t comm, int* cus) {
  if (!comm || !cus) return FTAR_ERR_INVALID_ARG;
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
ftar_status_t run_group(const void* const* sendbufs, void* const* recvbufs, size_t count, ftar_dtype_t dtype,
                        ftar_op_t op, const ftar_topo_t* topo, ftar_comm_t* comms, int nranks,
                        void* const* streams, bool host) {
  if (!recvbufs || !comms || nranks <= 0) return FTAR_ERR_INVALID_ARG;
  std::vector<ftar_status_t> st(nranks, FTAR_SUCCESS);
  std::vector<std::string> why(nranks);
  std::vector<std::thread> th;
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
  for (int r = 0; r < nranks; ++r)
    th.emplace_back([&, r] {
      hipStream_t s = streams ? static_cast<hipStream_t>(streams[r]) : nullptr;
      const void* sb = sendbufs ? sendbufs[r] : nullptr;
      if (capturing) comms[r]->tp->capture_enter();
      st[r] = host ? ftar_allreduce_host(sb, recvbufs[r], count, dtype, op, topo, comms[r], s)
                   : ftar::allreduce(sb, recvbufs[r], count, dtype, op, topo, comms[r], s);
      if (capturing) comms[r]->tp->capture_leave();
      if (!capturing && st[r] == FTAR_SUCCESS && hipSetDevice(comms[r]->device) == hipSuccess &&
          hipStreamSynchronize(s) != hipSuccess)
        st[r] = FTAR_ERR_HIP;
      if (st[r] != FTAR_SUCCESS) why[r] = ftar::last_error();  // the error text is per thread
    });
  for (auto& t : th) t.join();
  for (int r = 0; r < nranks; ++r)
    if (st[r] != FTAR_SUCCESS) {
      ftar::set_error("rank " + std::to_string(r) + ": " + why[r], __FILE__, __LINE__);  // to the caller's thread
      return st[r];
    }
  return FTAR_SUCCESS;
}
}  // namespace

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
