// C ABI: version/errors, the one-device reduce, topology parsing, the
// reference's cost model restated, and schedule introspection.  The xGMI
// execution model lives in cost_model.cpp; communicator and AllReduce entry
// points in engine.cpp.
#include <rccl/rccl.h>

#include <unistd.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <sstream>

#include <map>
#include "ftar_internal.h"

using ftar::hip_ignore;

namespace ftar {

namespace {
thread_local std::string g_last_error;
}

void set_error(const std::string& msg, const char* file, int line) {
  g_last_error = msg + " (" + file + ":" + std::to_string(line) + ")";
  if (getenv("FTAR_DEBUG")) fprintf(stderr, "[ftar] %s\n", g_last_error.c_str());
}
const char* last_error() { return g_last_error.c_str(); }

void trace(const char* fmt, ...) {
  static const bool on = getenv("FTAR_TRACE") && *getenv("FTAR_TRACE") && *getenv("FTAR_TRACE") != '0';
  if (!on) return;
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  fprintf(stderr, "[ftar pid %d] %s\n", (int)getpid(), buf);
  fflush(stderr);
}

namespace {

// ---------------------------------------------------------------------------
// The reference's cost model, restated (cost_model/CostModel.h:1-120), for
// FTAR_COST_MODEL=reference and for parity (tests/golden/costmodel.jsonl, the
// reference's own output).  Units are the reference's (undocumented; chunk =
// its Chunk_size, 100 in cost_model/main.cpp:23).  Same operations in the same
// order, so the doubles are the reference's bit for bit:
//   latency_control_overhead(100, w)  (CostModel.h:1-20; the chunk passed is
//                                      always 100, :92)
//   memory_read_write_overhead        (:32-79; height 1..9 only)
//   bandwidth_calculation_overhead    (:22-30)
// The first candidate's sum starts from an uninitialised `cost` there (:89);
// here from 0, which is what the reference's default (-O0) build prints.
// ---------------------------------------------------------------------------
double ref_latency(double chunk, double tw) {
  const double lo = 0.004, co = 0.0002;
  return tw > 9 ? 2 * lo + chunk * (tw - 9) * co : 2 * lo;
}

double ref_bandwidth(int total, double chunk) {
  const double bo = 0.0068, n = total;
  return (((n - 1) / n) * chunk) * bo;
}

// < 0: a height the reference has no case for (its switch falls off the end)
double ref_memory(const std::vector<int>& tree, int total, double chunk) {
  const int th = (int)tree.size();
  if (th < 1 || th > 9) return -1.0;
  const double o = 0.0004;
  // steps = n + 2*t0*..*t{h-2} + ... + 2*t0 + 1 (the switch's cases 1..9)
  int steps = total + 1, prod = 1;
  for (int i = 0; i + 1 < th; ++i) {
    prod *= tree[i];
    steps += 2 * prod;
  }
  return ((steps * chunk) / total) * o;
}

double ref_cost(const std::vector<int>& tree, int total, double chunk) {
  double mem = ref_memory(tree, total, chunk);
  if (mem < 0) return -1.0;
  double cost = 0;
  for (int w : tree) cost += ref_latency(100, w);
  cost += mem;
  cost += ref_bandwidth(total, chunk);
  return cost;
}

// getWidth(P) (GetWidth.h:10-47): ordered factorizations, smallest first
// factor first, the single factor [P] listed as [1,P], [P,1]
std::vector<std::vector<int>> ref_getwidth(int P) {
  std::vector<size_t> cur;
  std::vector<std::vector<size_t>> f;
  factorizations((size_t)P, cur, f);
  std::vector<std::vector<int>> out;
  for (auto& c : f) {
    if (c.size() == 1) {
      out.push_back({1, P});
      out.push_back({P, 1});
    } else {
      out.emplace_back(c.begin(), c.end());
    }
  }
  return out;
}

// a getWidth list as a topology: any width 1 selects the ring (mpi_mod.hpp:1440-1468)
void ref_list_topology(const std::vector<int>& w, ftar_topo_t* out) {
  memset(out, 0, sizeof *out);
  bool ring = false;
  for (int x : w) ring = ring || x == 1;
  if (ring) {
    out->ring = 1;
    out->nstages = 1;
    out->stages[0] = 1;
    return;
  }
  out->nstages = (int)std::min<size_t>(w.size(), FTAR_MAX_STAGES);
  for (int i = 0; i < out->nstages; ++i) out->stages[i] = w[i];
}

}  // namespace
}  // namespace ftar

extern "C" {

double ftar_cost_reference(const int* widths, int nwidths, int nranks, double chunk) {
  if (!widths || nwidths <= 0 || nranks <= 0) return -1.0;
  return ftar::ref_cost(std::vector<int>(widths, widths + nwidths), nranks, chunk);
}

ftar_status_t ftar_topo_choose_reference(int nranks, double chunk, ftar_topo_t* out, int* index) {
  if (!out || nranks <= 0) return FTAR_ERR_INVALID_ARG;
  if (nranks == 1) {  // getWidth(1) = one empty list the reference cannot score
    ftar::ref_list_topology({1}, out);
    if (index) *index = 0;
    return FTAR_SUCCESS;
  }
  const auto cands = ftar::ref_getwidth(nranks);
  double best = 1000000000;  // cost_output, CostModel.h:84
  int at = -1;
  for (size_t i = 0; i < cands.size(); ++i) {
    const double c = ftar::ref_cost(cands[i], nranks, chunk);
    if (c < 0) continue;
    if (c < best) {  // first minimum wins (:97)
      best = c;
      at = (int)i;
    }
  }
  if (at < 0) return FTAR_ERR_UNSUPPORTED;
  ftar::ref_list_topology(cands[at], out);
  if (index) *index = at;
  return FTAR_SUCCESS;
}

int ftar_cost_reference_candidates(int nranks, int* widths, int max_widths, int* lengths, int max_lists) {
  if (nranks <= 1) return -FTAR_ERR_INVALID_ARG;
  const auto cands = ftar::ref_getwidth(nranks);
  int used = 0;
  for (size_t i = 0; i < cands.size(); ++i) {
    if ((int)i < max_lists && lengths) lengths[i] = (int)cands[i].size();
    for (int w : cands[i]) {
      if (widths && used < max_widths) widths[used] = w;
      ++used;
    }
  }
  return (int)cands.size();
}

const char* ftar_version(void) {
  static char v[64];
  snprintf(v, sizeof v, "ftar %d.%d (gfx950)", FTAR_VERSION_MAJOR, FTAR_VERSION_MINOR);
  return v;
}

const char* ftar_status_string(ftar_status_t s) {
  switch (s) {
    case FTAR_SUCCESS: return "success";
    case FTAR_ERR_INVALID_ARG: return "invalid argument";
    case FTAR_ERR_UNSUPPORTED: return "unsupported (dtype/op, form or operation; see ftar_last_error)";
    case FTAR_ERR_INVALID_TOPO: return "invalid FT_TOPO/FT_LONELY";
    case FTAR_ERR_HIP: return "HIP error";
    case FTAR_ERR_RCCL: return "RCCL error";
    case FTAR_ERR_INTERNAL: return "internal error";
    case FTAR_ERR_TIMEOUT: return "timeout";
    case FTAR_ERR_NO_MEMORY: return "out of device memory";
  }
  return "unknown";
}

const char* ftar_last_error(void) { return ftar::last_error(); }

size_t ftar_dtype_size(ftar_dtype_t dt) { return ftar::dtype_size(dt); }

ftar_status_t ftar_reduce(const void* const* srcs, int k, void* dst, size_t count, ftar_dtype_t dtype, ftar_op_t op,
                          void* stream) {
  return ftar::launch_reduce(srcs, k, dst, count, dtype, op, static_cast<hipStream_t>(stream));
}

ftar_status_t ftar_reduce_nested(const void* const* srcs, int k, void* dst, size_t count, ftar_dtype_t dtype,
                                 ftar_op_t op, const int* shape, int nlevels, void* stream) {
  if (nlevels < 0 || nlevels > ftar::kMaxFoldLevels || (nlevels > 0 && !shape)) return FTAR_ERR_INVALID_ARG;
  if (nlevels > 1) {  // validate the shape for every dtype (only float sums use it)
    long long prod = 1;
    for (int l = 0; l < nlevels; ++l) {
      if (shape[l] < 1) return FTAR_ERR_INVALID_ARG;
      prod *= shape[l];
    }
    if (prod != k) return FTAR_ERR_INVALID_ARG;
  }
  return ftar::launch_reduce(srcs, k, dst, count, dtype, op, static_cast<hipStream_t>(stream), false, shape,
                             nlevels);
}

// get_stages (mpi_mod.hpp:1419-1486), minus its two bugs: an unset FT_TOPO
// is reported (the reference exit(1)s for every P > 1) and a trailing comma
// does not repeat the last width (the reference's `while(!ss.eof())` does).
ftar_status_t ftar_topo_parse(const char* ft_topo, const char* ft_lonely, int nranks, ftar_topo_t* out) {
  if (!out || nranks <= 0) return FTAR_ERR_INVALID_ARG;
  ftar_topo_t t{};
  if (ft_lonely && *ft_lonely) t.lonely = atoi(ft_lonely);
  if (!ft_topo || !*ft_topo) {
    // one rank and no lonely ranks: a copy (mpi_mod.hpp:1739-1746); reported as the ring, like any width 1.
    // The reference's check (:1471) takes the unset FT_TOPO as a product of 1, so FT_LONELY must be 0 here.
    if (nranks == 1 && t.lonely == 0) {
      t.nstages = 1;
      t.stages[0] = 1;
      t.ring = 1;
      *out = t;
      return FTAR_SUCCESS;
    }
    return FTAR_ERR_INVALID_TOPO;
  }
  std::string s(ft_topo);
  for (char& ch : s)
    if (ch == ',') ch = ' ';
  std::istringstream is(s);
  long w;
  while (is >> w) {
    if (t.nstages >= FTAR_MAX_STAGES || w <= 0) return FTAR_ERR_INVALID_TOPO;
    if (w == 1) {  // any 1 => ring
      ftar_topo_t r{};
      r.nstages = 1;
      r.stages[0] = 1;
      r.ring = 1;
      *out = r;
      return FTAR_SUCCESS;
    }
    t.stages[t.nstages++] = (int)w;
  }
  if (!is.eof() || t.nstages == 0) return FTAR_ERR_INVALID_TOPO;
  ftar::Topology chk;
  ftar_status_t st = ftar::to_topology(&t, nranks, &chk);
  if (st != FTAR_SUCCESS) return st;
  if (chk.lonely && ftar::check_world(chk, nranks, (size_t)nranks * 64, ftar::Form()) != FTAR_SUCCESS)
    return FTAR_ERR_INVALID_TOPO;  // a lonely layout the reference cannot run (its asserts / a blocked Waitall)
  *out = t;
  return FTAR_SUCCESS;
}

int ftar_topo_candidates(int nranks, ftar_topo_t* out, int max_out) {
  // the reference's getWidth(P) order (cost_model/GetWidth.h:10-47): ordered
  // factorizations, smallest first factor first; its {1,P}/{P,1} pair is the ring.
  if (nranks <= 0) return -FTAR_ERR_INVALID_ARG;
  std::vector<size_t> cur;
  std::vector<std::vector<size_t>> cands;
  ftar::factorizations((size_t)nranks, cur, cands);
  int n = 0;
  for (auto& c : cands) {
    ftar::Topology t;
    if (c.size() == 1) {  // the width-P single stage is listed as [1,P],[P,1] by the reference: ring first
      ftar::Topology r;
      r.ring = true;
      r.widths = {1};
      if (out && n < max_out) ftar::from_topology(r, &out[n]);
      ++n;
    }
    if (c.size() > FTAR_MAX_STAGES) continue;
    t.widths = c;
    if (out && n < max_out) ftar::from_topology(t, &out[n]);
    ++n;
  }
  return n;
}

ftar_status_t ftar_topo_from_env(int nranks, size_t bytes, ftar_topo_t* out) {
  // the engine's rule for topo == NULL (engine.cpp env_topology): both unset (FT_LONELY "0" = unset) ->
  // the cost model; anything else must parse, or it is reported
  const char* et = getenv("FT_TOPO");
  const char* el = getenv("FT_LONELY");
  if ((!et || !*et) && (!el || !*el || !strcmp(el, "0"))) return ftar_topo_choose(nranks, bytes, out);
  return ftar_topo_parse(et, el, nranks, out);
}

int ftar_topo_format(const ftar_topo_t* topo, char* buf, size_t buflen) {
  if (!topo) return -1;
  ftar::Topology t;
  std::string s;
  if (topo->ring) s = "ring";
  else {
    for (int i = 0; i < topo->nstages; ++i) s += (i ? "," : "") + std::to_string(topo->stages[i]);
    if (topo->lonely) s += "+" + std::to_string(topo->lonely);
  }
  if (buf && buflen) snprintf(buf, buflen, "%s", s.c_str());
  return (int)s.size();
}

ftar_status_t ftar_get_unique_id(ftar_unique_id_t* id) {
  if (!id) return FTAR_ERR_INVALID_ARG;
  static_assert(sizeof(ftar_unique_id_t) == sizeof(ncclUniqueId), "unique id size");
  ncclUniqueId u;
  ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) {
    ftar::set_error(std::string("ncclGetUniqueId: ") + ncclGetErrorString(r), __FILE__, __LINE__);
    return FTAR_ERR_RCCL;
  }
  memcpy(id, &u, sizeof(u));
  return FTAR_SUCCESS;
}

static long emit(const std::string& s, char* buf, size_t buflen) {
  if (buf && buflen) {
    size_t m = std::min(s.size(), buflen - 1);
    memcpy(buf, s.data(), m);
    buf[m] = 0;
  }
  return (long)s.size();
}

long ftar_schedule_json(const ftar_topo_t* topo, int nranks, int rank, size_t count, char* buf, size_t buflen) {
  ftar::Topology t;
  if (ftar::to_topology(topo, nranks, &t) != FTAR_SUCCESS) return -FTAR_ERR_INVALID_TOPO;
  std::string s;
  ftar_status_t st = ftar::schedule_json(t, nranks, rank, count, &s);
  if (st != FTAR_SUCCESS) return -(long)st;
  return emit(s, buf, buflen);
}

long ftar_plan_json(const ftar_topo_t* topo, int nranks, int rank, size_t count, ftar_allgather_t allgather,
                    ftar_reduce_scatter_t reduce_scatter, char* buf, size_t buflen) {
  ftar::Topology t;
  if (ftar::to_topology(topo, nranks, &t) != FTAR_SUCCESS) return -FTAR_ERR_INVALID_TOPO;
  ftar::Plan p;
  ftar::Form form;
  form.allgather = allgather;
  form.reduce_scatter = reduce_scatter;
  ftar_status_t st = ftar::build_plan(t, nranks, rank, count, &p, form);
  if (st != FTAR_SUCCESS) return -(long)st;
  return emit(p.json(), buf, buflen);
}

}  // extern "C"

// ---------------------------------------------------------------------------
// IPC primitives of the peer-direct transport, exported for tests (not part of
// ftar.h): the 2-process test maps one process's buffer into another on the
// same device and reduces through the mapping, as RcclTransport::map_peers does
// across devices.
// ---------------------------------------------------------------------------
// The reference is ftar::IpcRef (128 bytes): allocation handle + offset, so a
// pointer anywhere inside an allocation (a registered tensor) maps correctly.
namespace {
std::mutex g_dbg_mu;
std::map<void*, void*> g_dbg_bases;  // pointer handed out -> mapped allocation
}  // namespace

extern "C" ftar_status_t ftar_debug_ipc_handle(const void* ptr, void* ref128) {
  if (!ptr || !ref128) return FTAR_ERR_INVALID_ARG;
  ftar::IpcRef r;
  FTAR_RETURN_IF(ftar::ipc_export(ptr, &r));
  memcpy(ref128, &r, sizeof r);
  return FTAR_SUCCESS;
}

extern "C" ftar_status_t ftar_debug_ipc_open(const void* ref128, void** ptr) {
  if (!ref128 || !ptr) return FTAR_ERR_INVALID_ARG;
  ftar::IpcRef r;
  memcpy(&r, ref128, sizeof r);
  void* base = nullptr;
  char* p = nullptr;
  FTAR_RETURN_IF(ftar::ipc_import(r, &base, &p));
  std::lock_guard<std::mutex> g(g_dbg_mu);
  g_dbg_bases[p] = base;
  *ptr = p;
  return FTAR_SUCCESS;
}

extern "C" ftar_status_t ftar_debug_ipc_close(void* ptr) {
  if (!ptr) return FTAR_ERR_INVALID_ARG;
  void* base = ptr;
  {
    std::lock_guard<std::mutex> g(g_dbg_mu);
    auto it = g_dbg_bases.find(ptr);
    if (it != g_dbg_bases.end()) {
      base = it->second;
      g_dbg_bases.erase(it);
    }
  }
  FTAR_CHECK_HIP(hipIpcCloseMemHandle(base));
  return FTAR_SUCCESS;
}
