// Internal declarations of libftar (not part of the C ABI).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "ftar.h"

namespace ftar {

// A failed HIP call also leaves the thread's "last error" set, and the next
// kernel-launch check (hipGetLastError) would report it against an innocent
// launch: every failure path clears it once reported (clear_hip_error).
#define FTAR_CHECK_HIP(expr)                                                                   \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess) {                                                                    \
      ::ftar::set_error(std::string(#expr) + ": " + hipGetErrorString(_e), __FILE__, __LINE__); \
      (void)hipGetLastError();                                                                 \
      return FTAR_ERR_HIP;                                                                     \
    }                                                                                          \
  } while (0)

// best-effort HIP call (cleanup paths): a failure is dropped, and so is the
// sticky "last error" it would leave for the next launch check
// Device allocation: hipErrorOutOfMemory becomes FTAR_ERR_NO_MEMORY (so the MPI
// shim can answer MPI_ERR_NO_MEM), anything else FTAR_ERR_HIP.
#define FTAR_CHECK_ALLOC(expr)                                                                 \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess) {                                                                    \
      ::ftar::set_error(std::string(#expr) + ": " + hipGetErrorString(_e), __FILE__, __LINE__); \
      (void)hipGetLastError();                                                                 \
      return _e == hipErrorOutOfMemory ? FTAR_ERR_NO_MEMORY : FTAR_ERR_HIP;                    \
    }                                                                                          \
  } while (0)

inline void hip_ignore(hipError_t e) {
  if (e != hipSuccess) (void)hipGetLastError();
}

#define FTAR_RETURN_IF(st)          \
  do {                              \
    ftar_status_t _s = (st);        \
    if (_s != FTAR_SUCCESS) return _s; \
  } while (0)

void set_error(const std::string& msg, const char* file, int line);
// FTAR_TRACE=1: one stderr line per step of the collective bring-up paths
// (exchange-buffer growth, IPC export/import/close), so a stall names its call
void trace(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
const char* last_error();

// ---------------------------------------------------------------------------
// topology (mpi_mod.hpp:1419-1486)
// ---------------------------------------------------------------------------
struct Topology {
  std::vector<size_t> widths;  // bottom-up stage widths (tree); {1} for ring
  size_t lonely = 0;
  bool ring = false;
  std::string key() const;
};
ftar_status_t to_topology(const ftar_topo_t* t, int nranks, Topology* out);
void from_topology(const Topology& t, ftar_topo_t* out);

// ---------------------------------------------------------------------------
// the xGMI execution model (cost_model.cpp)
// ---------------------------------------------------------------------------
struct CostParams {  // seconds and bytes per second
  double alpha, link, hbm, issue, barrier, peer_read, peer_write, copy, coll;
};
CostParams cost_params();  // defaults <- calibration file <- ftar_cost_set <- FTAR_COST_* environment
uint64_t cost_generation();  // changes whenever the constants may have (cached choices expire)
// FTAR_COST_FILE's parse status (FTAR_SUCCESS when unset); a failure also sets the error text
ftar_status_t cost_file_status();
// every ordered factorization of n into factors >= 2 (cost_model/GetWidth.h:10-47)
void factorizations(size_t n, std::vector<size_t>& cur, std::vector<std::vector<size_t>>& out);
// the direct forms run it as one gather-and-fold round plus one all-gather round (schedule.cpp)
bool one_round_topology(const Topology& t, int P);
// predicted seconds; < 0 where the form cannot run this topology or its rate is unmeasured
double exec_cost(const Topology& t, int P, size_t bytes, int form, size_t chunk, bool registered,
                 const CostParams& k);
struct ExecChoice {
  Topology topo;
  int form = FTAR_FORM_DIRECT;
  size_t chunk = 0;  // 0: whole blocks
  double seconds = 0;
  int tied = 1;           // candidates priced equal to this one, itself included
  int tie_broken_by = 0;  // ftar_tie_t
};
// argmin over what `flags` (FTAR_CHOOSE_*) leaves free; the rest is fixed_*
ftar_status_t choose_exec(int P, size_t bytes, int flags, const Topology& fixed_topo, int fixed_form,
                          size_t fixed_chunk, ExecChoice* out);

// ---------------------------------------------------------------------------
// schedule (mpi_mod.hpp:80-766) lowered to an executable plan
// ---------------------------------------------------------------------------
enum BufId : int { BUF_SRC = 0, BUF_DST = 1, BUF_SCRATCH = 2 };

struct Transfer {
  int peer;
  int buf;     // BufId
  size_t off;  // elements into buf
  size_t len;  // elements (> 0)
};

struct Operand {
  int buf;     // BufId
  size_t off;  // element offset of this operand's copy of the block
};

struct ReduceItem {
  size_t off;                   // element offset of the block in dst
  size_t len;                   // elements (> 0)
  std::vector<Operand> srcs;    // fold order: dst = ((srcs[0] OP srcs[1]) OP srcs[2]) ...
  bool round_each = false;      // bf16: round after every add (one hop per add)
  std::vector<int> shape;       // nested fold of srcs (launch_reduce); empty = flat
};

struct Stage {
  std::vector<Transfer> sends, recvs;
  std::vector<ReduceItem> reduces;
};

struct Plan {
  int rank = 0, nranks = 1;
  size_t count = 0, split = 0;
  std::vector<Stage> stages;
  // forms actually used; COLLECTIVE = one all-gather of `split` elements at
  // r*split after the reduce-scatter stages
  int allgather = FTAR_AG_STAGES;
  int reduce_scatter = FTAR_RS_STAGES;
  size_t scratch_half = 0;  // elements per scratch half (stages alternate halves)
  int max_k = 0;
  std::string json() const;
};

// FMA-level schedule (for tests/introspection), JSON shaped like the reference dump.
ftar_status_t schedule_json(const Topology& t, int nranks, int rank, size_t count, std::string* out);
struct Form {
  int allgather = FTAR_AG_STAGES;
  int reduce_scatter = FTAR_RS_STAGES;
};
ftar_status_t build_plan(const Topology& t, int nranks, int rank, size_t count, Plan* out, Form form = Form());
// All ranks' plans pair up stage by stage (else FTAR_ERR_INVALID_TOPO).
ftar_status_t check_world(const Topology& t, int nranks, size_t count, Form form);

// ---------------------------------------------------------------------------
// reduce kernels (reduce_impl.h; dispatch in reduce_kernels.hip)
// ---------------------------------------------------------------------------
// srcs: host array of k device pointers. k == 1 copies.
// round_each: bf16 sums round to bf16 after every add (no effect on other dtypes).
// shape: bottom-up widths of a nested fold (srcs in depth-first leaf order,
// product == k, at most kMaxFoldLevels levels; bf16 inner nodes rounded);
// nlevels <= 1 = flat.  Only float sums depend on it: integer sums and AND are
// associative and take the flat kernel.
constexpr int kMaxFoldLevels = 4;
ftar_status_t launch_reduce(const void* const* srcs, int k, void* dst, size_t count, ftar_dtype_t dt, ftar_op_t op,
                            hipStream_t stream, bool round_each = false, const int* shape = nullptr,
                            int nlevels = 0, bool lds = true);
bool dtype_op_supported(ftar_dtype_t dt, ftar_op_t op);
// dst_i[0..bytes_i) = src_i[0..bytes_i) for up to FTAR_MAX_K segments in one
// launch (the peer-direct all-gather: each segment pulls one rank's block).
struct Segment {
  const void* src;
  void* dst;
  size_t bytes;
};
// nt: nontemporal loads and stores (the default: cold copies, data not
// re-read soon); false keeps both in the caches.  release_system: every
// workgroup ends with a system-scope release fence, so its stores are in
// memory before it retires (the host path's gather -> D2H hand-off).
ftar_status_t launch_gather(const Segment* segs, int nsegs, hipStream_t stream, bool nt = true,
                            size_t max_wg_per_seg = 0, bool release_system = false);
// launch_gather's launch for these segments: its workgroups, the segments with bytes (packed in order) and
// the bytes one workgroup copies per pass over a segment (workgroup w copies tiles w / nsegs + j * grid /
// nsegs of segment w % nsegs)
struct GatherGeom {
  unsigned grid = 0, nsegs = 0, tile_bytes = 0;
};
GatherGeom gather_geometry(const Segment* segs, int nsegs, size_t max_wg_per_seg);
// Diagnostic: launch_gather (no release) whose workgroups each leave a record when they end --
// 4 words in host_log, and a count of its runs and the XCDs they ran on in dev_log (2 words; reduce_impl.h
// gather_logged_kernel); cap_wg: records that fit
ftar_status_t launch_gather_logged(const Segment* segs, int nsegs, hipStream_t stream, bool nt,
                                   size_t max_wg_per_seg, unsigned* host_log, unsigned* dev_log, size_t cap_wg);
// An empty kernel: a stream-order point after the kernel before it (diagnostics).
ftar_status_t launch_noop(hipStream_t stream);
// One local device copy (k = 1 reduces, the P = 1 AllReduce, the peer forms' local copy-in/out): the
// LDS-staged kernel when source and destination share their 16-byte alignment, else the copy kernel.
ftar_status_t launch_copy(const void* src, void* dst, size_t bytes, hipStream_t stream);  // 0: enough workgroups for one pass
size_t dtype_size(ftar_dtype_t dt);

// ---------------------------------------------------------------------------
// transports (transport.cpp)
// ---------------------------------------------------------------------------
class Transport {
 public:
  virtual ~Transport() = default;
  virtual ftar_status_t group_start() = 0;
  virtual ftar_status_t send(const void* buf, size_t bytes, int peer, hipStream_t s) = 0;
  virtual ftar_status_t recv(void* buf, size_t bytes, int peer, hipStream_t s) = 0;
  virtual ftar_status_t group_end() = 0;
  virtual const char* name() const = 0;
  // All-gather of `bytes` per rank: rank r's segment at recv + r*bytes (in place
  // when send == recv + r*bytes).  Default: one group of p2p sends/receives.
  virtual ftar_status_t allgather(const void* send, void* recv, size_t bytes, int rank, int nranks, hipStream_t s) {
    FTAR_RETURN_IF(group_start());
    for (int p = 0; p < nranks; ++p)
      if (p != rank) FTAR_RETURN_IF(this->send(send, bytes, p, s));
    for (int p = 0; p < nranks; ++p)
      if (p != rank) FTAR_RETURN_IF(this->recv(static_cast<char*>(recv) + (size_t)p * bytes, bytes, p, s));
    return group_end();
  }
  // Peer-direct mode (engine.cpp peer_allreduce).  barrier: stream-ordered,
  // work after it on `s` starts once every rank's stream reached it.
  // map_peers: collective and host-blocking; every rank passes a pointer into
  // device memory (any offset into a hipMalloc allocation) and gets every
  // rank's pointer as an address usable by kernels on its own device
  // (peers[rank] == mine).  unmap_peers undoes it.
  virtual ftar_status_t barrier(hipStream_t s) = 0;
  // A barrier that also agrees on failures (the host transport's piece loop,
  // engine.cpp peer_allreduce_host): mine_ok says this rank's work since the
  // last barrier was issued without error, *all_ok that every rank's was, so
  // all ranks leave a failed call at the same barrier instead of some waiting
  // in the next one.  Default: the plain barrier, *all_ok = mine_ok.
  virtual ftar_status_t barrier_status(hipStream_t s, bool mine_ok, bool* all_ok) {
    *all_ok = mine_ok;
    return barrier(s);
  }
  // Host-synchronous agreement on `bytes` of per-call settings: *same = every
  // rank passed the same bytes.  Only the host transport's host-buffer path
  // needs it (the pipelined and whole-bucket paths run different numbers of
  // host barriers); elsewhere *same = true.
  virtual ftar_status_t agree(const void* mine, size_t bytes, bool* same) {
    (void)mine;
    (void)bytes;
    *same = true;
    return FTAR_SUCCESS;
  }
  // The first contact of a communicator (engine.cpp first_contact) may block the host inside the transport
  // library (RCCL: the settings all-gather and the p2p connection handshakes): the engine then runs it on a
  // helper thread it waits for with a deadline.  connect_peers makes every p2p connection now (collective);
  // abort stops the transport's in-flight work for good (ncclCommAbort), so a stuck helper returns.
  virtual bool first_contact_blocks() const { return false; }
  virtual ftar_status_t connect_peers(int rank) {
    (void)rank;
    return FTAR_SUCCESS;
  }
  virtual void abort() {}
  // RCCL user-buffer registration (ncclCommRegister, a local call): lets RCCL move p2p data straight
  // between registered buffers where it can.  Returns a handle, or nullptr where the transport has no
  // such registration or RCCL refused it (the transfers then take RCCL's staging path, same bytes).
  virtual void* rccl_register(void* buf, size_t bytes) {
    (void)buf;
    (void)bytes;
    return nullptr;
  }
  virtual void rccl_deregister(void* handle) { (void)handle; }
  virtual ftar_status_t map_peers(void* mine, int rank, int nranks, std::vector<char*>* peers) = 0;
  virtual void unmap_peers(std::vector<char*>* peers, int rank) { (void)rank; peers->clear(); }
  // map_peers exports and opens IPC handles (false: one address space)
  virtual bool uses_ipc() const { return false; }
  // send/recv are stream-ordered and need no peer participation beyond the
  // matching operation (RCCL, local).  false: the host transport, which has
  // no point-to-point transfers (peer-direct forms only).
  virtual bool async_p2p() const { return true; }
  // Stream capture of an in-process group (ftar_allreduce_group on capturing
  // streams): between enter and leave this thread issues its HIP calls only
  // while it holds the group's issue lock (released while it waits for a
  // peer), so the one capture graph is built by one host thread at a time.
  virtual void capture_enter() {}
  virtual void capture_leave() {}
  // A captured call issues serially on the caller's stream whatever the runtime (serial_capture, engine.cpp):
  // the in-process group.  Its ranks' forked comm/reduce streams, cross-waiting through the hub's events, make
  // HIP 7.2's hipStreamEndCapture recurse without end from P = 3 on (tools/capture/depth_probe.sh; P = 2
  // ends), while the serial form ends at every P, layout and piece size probed.
  virtual bool capture_serially() const { return false; }
  // The reduce stream may be a CU-masked one (ftar_comm_set_reduce_cus).  Not where the transport's kernels
  // wait on other processes on the device (RCCL): a masked stream takes a hardware queue of its own out of the
  // process's four and is a blocking stream, and over RCCL that stalled ranks in a call.
  virtual bool masked_reduce_stream_ok() const { return true; }
  // Called by every rank before it joins its internal streams back into the
  // caller's stream.  Under capture the local transport makes the ranks meet
  // here first: HIP's capture breaks (hipStreamEndCapture recurses without
  // end, tools/capture/) when a stream waits on an event of a stream that was
  // already joined back into its parent -- a peer's last wait on my "copied"
  // event must come before my join.
  virtual ftar_status_t before_join() { return FTAR_SUCCESS; }
  // The transport library's own collective, for comparison (RCCL only).
  virtual ftar_status_t native_allreduce(const void* send, void* recv, size_t count, ftar_dtype_t dt, ftar_op_t op,
                                         hipStream_t s) {
    (void)send; (void)recv; (void)count; (void)dt; (void)op; (void)s;
    return FTAR_ERR_UNSUPPORTED;
  }
};

// IPC reference to any device pointer: the handle of its allocation plus the
// pointer's offset in it (dmabuf IPC exports whole allocations).
struct IpcRef {
  hipIpcMemHandle_t handle;
  uint64_t offset;
  uint64_t valid;     // 1 when the export succeeded: peers never open a failed rank's handle
  uint64_t size;      // the exported allocation's size
  uint64_t stamped;   // 1: the first 16 bytes at the pointer are a fresh random token (stamp_token);
                      // 2: they are a caller's buffer's current content (registration) ...
  uint64_t token[2];  // ... and this is their value; the importer reads them back through its mapping
  uint64_t pad[2];
};
static_assert(sizeof(IpcRef) == 128, "IpcRef layout");
// On failure *out is still a well-formed reference with valid = 0, so the
// caller publishes it like any other and every rank learns of the failure in
// the same exchange (an unpublished or garbage handle would leave the peers
// blocked in hipIpcOpenMemHandle or in the exchange itself).
ftar_status_t ipc_export(const void* p, IpcRef* out);
// HIP runtimes before 7.2 (torch 2.10 bundles 7.0) block forever in
// hipIpcOpenMemHandle when the exported allocation's size has bit 31 set
// (2-4 GiB, 6-8 GiB, ...; measured: tools/ipc_order_probe.py --torch).  When
// the loaded runtime is affected (or FTAR_IPC_SIZE_GUARD=1; =0 turns it off)
// ipc_export refuses such allocations and the exchange buffers are sized
// around them (ipc_safe_size).
bool ipc_size_guard();
size_t ipc_safe_size(size_t bytes);
// A device buffer of `bytes` for IPC export (ipc = true: rounded by
// ipc_safe_size and export-checked; an allocation whose export fails -- a
// fresh hipMalloc landing on a recently closed IPC mapping can -- is set aside
// and another taken).  *out = nullptr on failure, with the error set: callers
// in a collective still publish (an invalid reference) so every rank fails
// together.  *got = the size allocated.
ftar_status_t alloc_exportable(size_t bytes, bool ipc, void** out, size_t* got);
// Writes a fresh random token into the first 16 bytes at p (a buffer ftar
// owns), so that its IPC reference can be verified by every importer: under
// HIP 7.0 an import occasionally maps the wrong memory after buffers were
// regrown (round-1 multi-process rehearsals on one GPU), silently.
ftar_status_t stamp_token(void* p);
void forget_token(const void* p);  // before the stamped buffer is freed
// opens ref and verifies the mapping (allocation size; the token when
// stamped) -- a mismatch closes it and fails like a failed open;
// *base = the mapped allocation (for hipIpcCloseMemHandle), *p = base + offset
ftar_status_t ipc_import(const IpcRef& ref, void** base, char** p);

std::unique_ptr<Transport> make_rccl_transport(int nranks, const ftar_unique_id_t& id, int rank,
                                               ftar_status_t* st);
struct LocalHub;
std::shared_ptr<LocalHub> make_local_hub(int nranks);
std::unique_ptr<Transport> make_local_transport(std::shared_ptr<LocalHub> hub, int rank);
std::unique_ptr<Transport> make_host_transport(int nranks, int rank, ftar_host_allgather_fn fn, void* user);

}  // namespace ftar
