// The communicator's state and the engine's interfaces between its translation units (not the C ABI):
//   engine.cpp       communicator lifecycle and settings, the two-stream executor
//   engine_api.cpp   the C ABI (bring-up, setters, entry points, in-process group calls)
//   engine_peer.cpp  the peer-direct forms (IPC-mapped exchange buffers over xGMI) and the xGMI probe
//   engine_host.cpp  host buffers on a host-bootstrapped communicator, the piece-pipelined read form
#pragma once

#include <condition_variable>
#include <cstdint>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "ftar_internal.h"

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
  // FTAR_DEBUG_HOST_GATHER_LOG (diagnostic, engine_host.cpp): one record per gather workgroup of
  // the last host-path call (launch_gather_logged), and each piece's launch geometry
  struct GatherLog {
    unsigned* host = nullptr;  // pinned host memory, 4 words per workgroup
    unsigned* dev = nullptr;   // device memory, 2 words per workgroup: how many times it ran, on which XCDs
    size_t cap = 0;            // workgroups both hold
    struct Piece {
      size_t first;            // the piece's first record
      ftar::GatherGeom geom;
      size_t off[FTAR_MAX_K], bytes[FTAR_MAX_K];  // each segment's destination, bytes from the exchange buffer
    };
    std::vector<Piece> pieces;
  } glog;
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

// phase timing (ftar_comm_set_phase_timing): one timing event at a phase boundary, on the stream reaching it
ftar_status_t mark(ftar_comm* c, const std::string& name, hipStream_t s);
// the call's event pool holds at least n events (a captured call gets a fresh set)
ftar_status_t grow_events(ftar_comm* c, size_t n);
// FTAR_ERR_UNSUPPORTED (with a message) when a buffer would grow under stream capture
ftar_status_t refuse_growth_under_capture(const ftar_comm* c, const char* what);

// ---- engine.cpp -----------------------------------------------------------------------------------------
// Host mode piece per block: 0 = auto (auto_host_chunk)
constexpr size_t kDefaultHostChunkBytes = 0;
// host mode (p2p transports): H2D pieces issued ahead of the step that first reads them
constexpr size_t kHostLookahead = 2;
// host mode on a host-bootstrapped communicator (peer_allreduce_host): H2D pieces issued ahead of the fold
// that reads them (the host waits at a barrier after every fold)
constexpr size_t kHostPeerLookahead = 3;
struct HostIO;
// bring-up of a communicator whose transport is set (streams, settings from the environment; a
// host-bootstrapped one agrees on them here), and its teardown (false: it must not be freed)
ftar_status_t comm_setup(ftar_comm* c);
bool comm_teardown(ftar_comm* c);
// one call on a communicator (device buffers, or host ones when `host` is set)
ftar_status_t allreduce(const void* sendbuf, void* recvbuf, size_t count, ftar_dtype_t dt, ftar_op_t op,
                        const ftar_topo_t* topo, ftar_comm* c, hipStream_t stream, const HostIO* host = nullptr);
// the reduce stream on `cus` CUs (0 = all); refused on RCCL communicators
ftar_status_t set_reduce_cus(ftar_comm* c, int cus);
// the form the explicit settings describe (ftar_form_t), or -2; set_form applies one
int form_of(const ftar_comm* c);
void set_form(ftar_comm* c, int form);

// ---- engine_peer.cpp ------------------------------------------------------------------------------------
// a one-round plan the peer kernels can run (one block per peer each way, all-gather straight into recvbuf)
bool peer_eligible(const Plan& plan);
// the exchange buffer X: grow-only, exported and mapped by every rank (collective)
ftar_status_t ensure_xbuf(ftar_comm* c, size_t bytes);
// where operand i of my block's fold lives: (the rank whose copy it is, -1 = mine; element offset) -> address
using OperandAt = std::function<const void*(int, size_t)>;
// the plan's fold of my block with its operands read from where(); elements [lo, lo + len) of the block only
ftar_status_t peer_fold(const ReduceItem& r, const Plan& plan, ftar_dtype_t dt, ftar_op_t op, void* dst,
                        hipStream_t s, bool lds, const OperandAt& where, size_t lo = 0, size_t len = SIZE_MAX);
// the cross-GPU copies of the peer forms: one copy-kernel launch over every segment, or DMA copies
ftar_status_t peer_copy(ftar_comm* c, const std::vector<Segment>& segs);
ftar_status_t peer_allreduce(const void* sendbuf, void* recvbuf, size_t count, ftar_dtype_t dt, ftar_op_t op,
                             const Plan& plan, ftar_comm* c, hipStream_t stream, int mode);
ftar_status_t xgmi_probe(ftar_comm* c, size_t bytes, int iters, double* out, int nout, size_t max_wg_per_seg);

// ---- engine_host.cpp ------------------------------------------------------------------------------------
// Host mode: sendbuf/recvbuf of the call are host memory (pinned for overlap).
struct HostIO {
  const char* src;
  char* dst;
};
// elements per piece of peer_allreduce_host
size_t host_peer_piece(const ftar_comm* c, size_t split, size_t esz);
ftar_status_t peer_allreduce_host(const HostIO& io, size_t count, ftar_dtype_t dt, ftar_op_t op, const Plan& plan,
                                  ftar_comm* c, hipStream_t stream);

}  // namespace ftar
