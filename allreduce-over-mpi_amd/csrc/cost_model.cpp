// The xGMI execution model: (topology, data-movement form, pipeline piece) for one MI355X node.
//
// Role of the reference's cost model (cost_model/CostModel.h:82-120: score every getWidth(P) width list
// for a chunk size, take the argmin).  That model charges a 16-host MPI cluster's per-layer latency and
// memory steps; it never sees that a tree stage of width w talks to w-1 peers AT ONCE, nor that the data
// moves in pieces whose fold overlaps the next piece's transfer.  On an MI355X node every peer is its own
// xGMI link, and with the one-round forms (schedule.cpp) every topology moves exactly tree(P)'s bytes, so
// what actually varies is HOW the bytes move (the form) and in what PIECES.  This model prices both:
//
//   per piece of a round:  r(x) = max(alpha + x / link, issue)     x = bytes one link carries per piece
//   fold of a piece:       f = (k + 1) * c / hbm                     k sources, c bytes each (reduce stream)
//   the two streams:       piece k's fold waits for its transfer, the next round's piece k waits for its fold
//                          (engine.cpp: ev_x / ev_r); simulated piece by piece, so fill and drain and
//                          per-piece overhead trade off against each other (small pieces pay m * alpha and
//                          m * issue, large ones leave the last fold exposed)
//   peer forms (no pieces): barriers, one pass of xGMI loads or stores per round, the fold, and the local
//                          copy-in (read) or copy-out (write) unless the buffers are registered
//   collective all-gather: alpha + (P - 1) * B / coll
//
// alpha, link, hbm, issue, barrier, peer read/write, copy and coll are constants of the node: defaults
// below, ftar_cost_set (bench.py fits them from ftar_xgmi_probe and from the sweep's own timings), and the
// environment over both.  Forms whose rate is unmeasured (peer forms, the collective) are never chosen.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <tuple>

#include "ftar_internal.h"

namespace ftar {

namespace {
std::mutex g_cost_mu;
ftar_cost_params_t g_set{};   // fields <= 0: default
ftar_cost_params_t g_loaded{};   // constants from ftar_cost_load
ftar_cost_params_t g_envfile{};  // constants from the file FTAR_COST_FILE names (kept apart: clearing the
                                 // variable drops these and leaves an explicit load in effect)
std::atomic<uint64_t> g_generation{0};  // bumped by every set: communicators re-decide their cached choices

// MI355X defaults, used where no run on the node has fitted them (bench.py at N > 1 does):
//   alpha   one p2p group's launch and handshake (assumed, 20 us)
//   link    an RCCL p2p stream to one peer: the xGMI link spec, 76.8 GB/s per direction, times an ASSUMED
//           RCCL p2p efficiency of 0.7 (protocol and FIFO staging; never measured on xGMI here -- the first
//           N > 1 run's probe and sweep replace it)
//   hbm     the measured k = 2..8 fold (profiles/r01/kbench3)
//   issue   the host enqueue of one piece of one round at P = 8 (enqueue cost)
//   barrier a 4-byte ncclAllReduce (assumed)
//   copy    the LDS-staged copy (profiles/r03/kbench_copy.log)
//   peer read / write, coll: unmeasured (0), so those forms are never chosen until a run measures them
constexpr double kXgmiLinkSpecGBps = 76.8, kRcclP2pEfficiency = 0.7;
constexpr ftar_cost_params_t kDefaults = {20.0, kXgmiLinkSpecGBps * kRcclP2pEfficiency, 6300.0, 25.0, 20.0,
                                          0.0,  0.0,                                      6500.0, 0.0};

double env_or(const char* name, double v) {
  const char* e = getenv(name);
  return e && *e ? atof(e) : v;
}

// The fields of ftar_cost_params_t by name, in struct order (the calibration file's keys)
constexpr const char* kFieldNames[9] = {"alpha_us",       "link_gbps",       "hbm_gbps",  "issue_us", "barrier_us",
                                        "peer_read_gbps", "peer_write_gbps", "copy_gbps", "coll_gbps"};
double* field(ftar_cost_params_t* p, int i) { return &p->alpha_us + i; }
static_assert(sizeof(ftar_cost_params_t) == 9 * sizeof(double), "ftar_cost_params_t is nine doubles");

// A calibration file: one "name value" (or "name = value") per line, '#' starts a comment; the names are
// ftar_cost_params_t's fields, every value a number > 0; fields left out keep their defaults.
ftar_status_t parse_cost_file(const char* path, ftar_cost_params_t* out) {
  FILE* f = fopen(path, "r");
  if (!f) {
    set_error(std::string("cost file ") + path + ": cannot open", __FILE__, __LINE__);
    return FTAR_ERR_INVALID_ARG;
  }
  ftar_cost_params_t p{};
  char line[512];
  int lineno = 0;
  ftar_status_t st = FTAR_SUCCESS;
  while (st == FTAR_SUCCESS && fgets(line, sizeof line, f)) {
    ++lineno;
    if (char* h = strchr(line, '#')) *h = 0;
    for (char* q = line; *q; ++q)
      if (*q == '=') *q = ' ';
    char name[128];
    double v = 0;
    char extra[8];
    const int got = sscanf(line, "%127s %lf %7s", name, &v, extra);
    if (got <= 0) continue;  // blank or comment
    int i = 0;
    while (i < 9 && strcmp(name, kFieldNames[i])) ++i;
    if (got != 2 || i == 9 || !(v > 0) || !std::isfinite(v)) {
      set_error(std::string("cost file ") + path + " line " + std::to_string(lineno) +
                    ": expected '<field> <value > 0>' with a field of ftar_cost_params_t",
                __FILE__, __LINE__);
      st = FTAR_ERR_INVALID_ARG;
    } else {
      *field(&p, i) = v;
    }
  }
  fclose(f);
  if (st == FTAR_SUCCESS) *out = p;
  return st;
}

// FTAR_COST_FILE: read at the first use of the model constants after the variable changes.  A file that
// parses replaces the previous file's constants; one that does not leaves them as they were (it is parsed
// into a temporary) and fails the next communicator bring-up (cost_file_status); an unset variable drops
// the file's constants and leaves ftar_cost_load's in effect.
std::string g_file_path;
ftar_status_t g_file_status = FTAR_SUCCESS;
std::string g_file_error;
void sync_cost_file() {  // under g_cost_mu
  const char* e = getenv("FTAR_COST_FILE");
  const std::string path = e ? e : "";
  if (path == g_file_path) return;
  g_file_path = path;
  g_file_status = FTAR_SUCCESS;
  if (path.empty()) {
    g_envfile = ftar_cost_params_t{};
  } else {
    ftar_cost_params_t p;
    g_file_status = parse_cost_file(path.c_str(), &p);
    if (g_file_status == FTAR_SUCCESS) g_envfile = p;
    else g_file_error = last_error();
  }
  ++g_generation;
}
}  // namespace

uint64_t cost_generation() {
  std::lock_guard<std::mutex> g(g_cost_mu);
  sync_cost_file();
  return g_generation.load();
}

ftar_status_t cost_file_status() {
  std::lock_guard<std::mutex> g(g_cost_mu);
  sync_cost_file();
  if (g_file_status != FTAR_SUCCESS) set_error("FTAR_COST_FILE: " + g_file_error, __FILE__, __LINE__);
  return g_file_status;
}

// precedence: FTAR_COST_<FIELD> > ftar_cost_set > FTAR_COST_FILE's file > ftar_cost_load's > the defaults
CostParams cost_params() {
  ftar_cost_params_t p, fp;
  {
    std::lock_guard<std::mutex> g(g_cost_mu);
    sync_cost_file();
    p = g_set;
    fp = g_loaded;
    for (int i = 0; i < 9; ++i)
      if (*field(&g_envfile, i) > 0) *field(&fp, i) = *field(&g_envfile, i);
  }
  auto pick = [](double set, double file, double def) { return set > 0 ? set : file > 0 ? file : def; };
  CostParams k;
  k.alpha = env_or("FTAR_COST_ALPHA_US", pick(p.alpha_us, fp.alpha_us, kDefaults.alpha_us)) * 1e-6;
  k.link = env_or("FTAR_COST_LINK_GBPS", pick(p.link_gbps, fp.link_gbps, kDefaults.link_gbps)) * 1e9;
  k.hbm = env_or("FTAR_COST_HBM_GBPS", pick(p.hbm_gbps, fp.hbm_gbps, kDefaults.hbm_gbps)) * 1e9;
  k.issue = env_or("FTAR_COST_ISSUE_US", pick(p.issue_us, fp.issue_us, kDefaults.issue_us)) * 1e-6;
  k.barrier = env_or("FTAR_COST_BARRIER_US", pick(p.barrier_us, fp.barrier_us, kDefaults.barrier_us)) * 1e-6;
  k.peer_read =
      env_or("FTAR_COST_PEER_READ_GBPS", pick(p.peer_read_gbps, fp.peer_read_gbps, kDefaults.peer_read_gbps)) * 1e9;
  k.peer_write =
      env_or("FTAR_COST_PEER_WRITE_GBPS", pick(p.peer_write_gbps, fp.peer_write_gbps, kDefaults.peer_write_gbps)) *
      1e9;
  k.copy = env_or("FTAR_COST_COPY_GBPS", pick(p.copy_gbps, fp.copy_gbps, kDefaults.copy_gbps)) * 1e9;
  k.coll = env_or("FTAR_COST_COLL_GBPS", pick(p.coll_gbps, fp.coll_gbps, kDefaults.coll_gbps)) * 1e9;
  return k;
}

void factorizations(size_t n, std::vector<size_t>& cur, std::vector<std::vector<size_t>>& out) {
  if (n == 1) {
    if (!cur.empty()) out.push_back(cur);
    return;
  }
  for (size_t f = 2; f <= n; ++f)
    if (n % f == 0) {
      cur.push_back(f);
      factorizations(n / f, cur, out);
      cur.pop_back();
    }
}

bool one_round_topology(const Topology& t, int P) {  // schedule.cpp: the direct forms run it in one round
  if (P > FTAR_MAX_K) return false;
  if (t.ring) return true;
  return t.lonely == 0 && t.widths.size() <= (size_t)kMaxFoldLevels;
}

namespace {

// One round structure of the two-stream pipeline: `rounds` consecutive rounds of m pieces on the comm
// stream; round j's piece k waits for the fold of the latest folding round's piece k (fold[j] > 0: round j
// is followed by a fold of f seconds per piece).  Returns the finish time of the last piece of the last
// round and of the last fold.
double pipeline(const std::vector<double>& r, const std::vector<double>& fold, size_t m) {
  // comm: c = end of the previous piece on the comm stream; red: end of the previous fold
  std::vector<double> last_fold(m, 0.0);  // end of the latest fold of piece k
  double comm = 0.0, red = 0.0;
  for (size_t j = 0; j < r.size(); ++j) {
    for (size_t k = 0; k < m; ++k) {
      comm = std::max(comm, last_fold[k]) + r[j];
      if (fold[j] > 0) {
        red = std::max(red, comm) + fold[j];
        last_fold[k] = red;
      }
    }
  }
  return std::max(comm, red);
}

// rounds of a staged tree's reduce-scatter: per stage, the bytes one link carries per piece of c (blocks
// per partner x c) and the fold's sources
void staged_tree_rounds(const Topology& t, int P, double c, const CostParams& k, std::vector<double>* r,
                        std::vector<double>* f) {
  double prod = 1;
  std::vector<double> per_link;
  for (size_t w : t.widths) {
    prod *= (double)w;
    const double blocks = (double)P / prod;  // blocks each partner receives per stage (the group's share)
    per_link.push_back(blocks * c);
    r->push_back(std::max(k.alpha + blocks * c / k.link, k.issue));
    f->push_back((double)(w + 1) * blocks * c / k.hbm);
  }
  for (size_t s = per_link.size(); s-- > 0;) {  // the all-gather stages, reversed, no folds
    r->push_back(std::max(k.alpha + per_link[s] / k.link, k.issue));
    f->push_back(0.0);
  }
}

}  // namespace

double exec_cost(const Topology& t, int P, size_t bytes, int form, size_t chunk, bool registered,
                 const CostParams& k) {
  if (P <= 1 || bytes == 0) return 0.0;
  const double S = (double)bytes, B = std::ceil(S / P);
  const bool peer = form == FTAR_FORM_PEER_READ || form == FTAR_FORM_PEER_WRITE;
  if (peer) {
    // the peer forms run one-round plans only (engine.cpp peer_eligible), whole blocks per kernel
    if (!one_round_topology(t, P) && !(t.lonely == 0 && t.widths.size() == 1)) return -1.0;
    const double fold = (double)(P + 1) * B / k.hbm;
    if (form == FTAR_FORM_PEER_READ) {
      if (k.peer_read <= 0) return -1.0;
      const double copy_in = registered ? 0.0 : 2.0 * S / k.copy;
      return 3.0 * k.barrier + copy_in + std::max(B / k.peer_read, fold) + B / k.peer_read;
    }
    if (k.peer_write <= 0) return -1.0;
    // unregistered outputs: the copy-out of the final blocks, and a third barrier after it (engine.cpp)
    const double copy_out = registered ? 0.0 : 2.0 * (P - 1) * B / k.copy + k.barrier;
    return 2.0 * k.barrier + 2.0 * B / k.peer_write + fold + copy_out;
  }
  const double c = chunk ? std::min<double>((double)chunk, B) : B;
  const size_t m = (size_t)std::max(1.0, std::ceil(B / c));
  const double rp = std::max(k.alpha + c / k.link, k.issue);  // one piece on every link at once
  std::vector<double> r, f;
  // the staged reduce-scatter rounds: the ring's P-1 neighbour steps (2-source folds) or a tree's stages
  auto staged_rs = [&] {
    if (t.ring) {
      for (int s = 0; s < P - 1; ++s) {
        r.push_back(rp);
        f.push_back(3.0 * c / k.hbm);
      }
      return;
    }
    staged_tree_rounds(t, P, c, k, &r, &f);
    r.resize(t.widths.size());  // the reduce-scatter half
    f.resize(t.widths.size());
    if (t.lonely) {  // the lonely ranks' data in
      r.push_back(rp);
      f.push_back(0.0);
    }
  };
  if (form == FTAR_FORM_DIRECT || form == FTAR_FORM_COLLECTIVE) {
    const bool single = !t.ring && t.lonely == 0 && t.widths.size() == 1;
    if (t.lonely == 0 && (one_round_topology(t, P) || single)) {
      r.push_back(rp);  // one gather round, one k = P fold per piece
      f.push_back((double)(P + 1) * c / k.hbm);
    } else {  // lonely layouts, trees deeper than the fold kernel, rings wider than one reduce: staged
      staged_rs();
    }
    if (form == FTAR_FORM_COLLECTIVE) {
      if (k.coll <= 0 || t.ring || t.lonely) return -1.0;  // ring / lonely: the engine falls back to direct
      return pipeline(r, f, m) + k.alpha + (P - 1) * B / k.coll;
    }
    r.push_back(rp);  // the direct all-gather: one round on every link
    f.push_back(0.0);
    if (t.lonely) {  // the lonely ranks' results out
      r.push_back(rp);
      f.push_back(0.0);
    }
    return pipeline(r, f, m);
  }
  if (form != FTAR_FORM_STAGES) return -1.0;
  if (t.ring) {  // 2(P-1) neighbour steps on one link each
    staged_rs();
    for (int s = 0; s < P - 1; ++s) {
      r.push_back(rp);
      f.push_back(0.0);
    }
    return pipeline(r, f, m);
  }
  staged_tree_rounds(t, P, c, k, &r, &f);
  if (t.lonely) {
    r.insert(r.begin() + (long)t.widths.size(), rp);
    f.insert(f.begin() + (long)t.widths.size(), 0.0);
    r.push_back(rp);
    f.push_back(0.0);
  }
  return pipeline(r, f, m);
}

ftar_status_t choose_exec(int P, size_t bytes, int flags, const Topology& fixed_topo, int fixed_form,
                          size_t fixed_chunk, ExecChoice* out) {
  const CostParams k = cost_params();
  std::vector<Topology> topos;
  if (flags & FTAR_CHOOSE_TOPO) {
    std::vector<size_t> cur;
    std::vector<std::vector<size_t>> cands;
    factorizations((size_t)P, cur, cands);
    for (auto& c : cands) {
      if (c.size() > FTAR_MAX_STAGES) continue;
      bool fits = true;  // one stage folds w sources: at most FTAR_MAX_K (engine.cpp)
      for (size_t w : c) fits = fits && w <= FTAR_MAX_K;
      if (!fits) continue;
      Topology t;
      t.widths = c;
      topos.push_back(t);
    }
    Topology ring;
    ring.ring = true;
    ring.widths = {1};
    topos.push_back(ring);
  } else {
    topos.push_back(fixed_topo);
  }
  std::vector<int> forms;
  if (flags & FTAR_CHOOSE_FORM) {
    forms = {FTAR_FORM_DIRECT, FTAR_FORM_STAGES, FTAR_FORM_COLLECTIVE};
    if (flags & FTAR_CHOOSE_PEER) {
      forms.push_back(FTAR_FORM_PEER_READ);
      forms.push_back(FTAR_FORM_PEER_WRITE);
    }
  } else {
    forms.push_back(fixed_form);
  }
  std::vector<size_t> chunks;
  if (flags & FTAR_CHOOSE_CHUNK) {
    for (size_t c = 256u << 10; c <= (256u << 20); c *= 2) chunks.push_back(c);
    chunks.push_back(0);  // whole blocks
  } else {
    chunks.push_back(fixed_chunk);
  }
  bool found = false;
  ExecChoice best;
  best.seconds = 0;
  const double B = std::ceil((double)bytes / std::max(1, P));
  const bool whole = std::find(chunks.begin(), chunks.end(), (size_t)0) != chunks.end();
  // ties (within 1e-9): the fewest stages (the ring last: the flat fold rounds bf16 once), then the form in
  // enum order (the simpler data movement), then the larger piece (fewer groups)
  auto tie_key = [&](const Topology& t, int form, size_t c) {
    const size_t stages = t.ring ? (size_t)P : t.widths.size() + (t.lonely ? 2 : 0);
    return std::make_tuple(stages, form, c == 0 ? size_t(0) : ~c);  // smaller wins; whole blocks (0) first
  };
  struct Priced {
    Topology t;
    int form;
    size_t chunk;
    double s;
  };
  std::vector<Priced> priced;
  for (const Topology& t : topos)
    for (int form : forms) {
      const bool peer = form == FTAR_FORM_PEER_READ || form == FTAR_FORM_PEER_WRITE;
      for (size_t c : chunks) {
        if (peer && c != chunks.front()) continue;  // the peer forms move whole blocks
        if (whole && c && (double)c >= B) continue;  // the same as whole blocks
        const double s = exec_cost(t, P, bytes, form, peer ? 0 : c, false, k);
        if (s < 0) continue;
        priced.push_back({t, form, peer ? (size_t)0 : c, s});
        const bool better = !found || s < best.seconds * (1 - 1e-9) ||
                            (s <= best.seconds * (1 + 1e-9) &&
                             tie_key(t, form, peer ? 0 : c) < tie_key(best.topo, best.form, best.chunk));
        if (better) {
          found = true;
          best.topo = t;
          best.form = form;
          best.chunk = peer ? 0 : c;
          best.seconds = s;
        }
      }
    }
  if (!found) {
    set_error("the execution model has no runnable choice for this topology / form", __FILE__, __LINE__);
    return FTAR_ERR_UNSUPPORTED;
  }
  // the tie, said out loud: how many candidates the model priced alike, and the highest-ranked tie rule that
  // set the choice apart from one of them (stages before form before piece)
  const auto bk = tie_key(best.topo, best.form, best.chunk);
  best.tied = 0;
  best.tie_broken_by = FTAR_TIE_NONE;
  for (const Priced& q : priced) {
    if (std::fabs(q.s - best.seconds) > best.seconds * 1e-9) continue;
    ++best.tied;
    const auto qk = tie_key(q.t, q.form, q.chunk);
    if (qk == bk) continue;
    const int rule = std::get<0>(qk) != std::get<0>(bk)   ? FTAR_TIE_STAGES
                     : std::get<1>(qk) != std::get<1>(bk) ? FTAR_TIE_FORM
                                                          : FTAR_TIE_PIECE;
    if (best.tie_broken_by == FTAR_TIE_NONE || rule < best.tie_broken_by) best.tie_broken_by = rule;
  }
  *out = best;
  return FTAR_SUCCESS;
}

}  // namespace ftar

extern "C" {

ftar_status_t ftar_cost_set(const ftar_cost_params_t* p) {
  if (!p) return FTAR_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(ftar::g_cost_mu);
  ftar::g_set = *p;
  ++ftar::g_generation;
  return FTAR_SUCCESS;
}

ftar_status_t ftar_cost_load(const char* path) {
  ftar_cost_params_t p{};  // path == NULL: forget the loaded constants
  if (path) FTAR_RETURN_IF(ftar::parse_cost_file(path, &p));
  std::lock_guard<std::mutex> g(ftar::g_cost_mu);
  ftar::g_loaded = p;
  ++ftar::g_generation;
  return FTAR_SUCCESS;
}

ftar_status_t ftar_cost_save(const char* path) {
  if (!path) return FTAR_ERR_INVALID_ARG;
  ftar_cost_params_t p;
  FTAR_RETURN_IF(ftar_cost_get(&p));
  FILE* f = fopen(path, "w");
  if (!f) {
    ftar::set_error(std::string("ftar_cost_save: cannot write ") + path, __FILE__, __LINE__);
    return FTAR_ERR_INVALID_ARG;
  }
  fprintf(f, "# ftar execution-model constants (ftar_cost_save; load with FTAR_COST_FILE or ftar_cost_load)\n");
  for (int i = 0; i < 9; ++i)
    if (*ftar::field(&p, i) > 0) fprintf(f, "%s %.15g\n", ftar::kFieldNames[i], *ftar::field(&p, i));
  const bool ok = fclose(f) == 0;
  if (!ok) ftar::set_error(std::string("ftar_cost_save: write failed: ") + path, __FILE__, __LINE__);
  return ok ? FTAR_SUCCESS : FTAR_ERR_INVALID_ARG;
}

ftar_status_t ftar_cost_get(ftar_cost_params_t* p) {
  if (!p) return FTAR_ERR_INVALID_ARG;
  const ftar::CostParams k = ftar::cost_params();
  p->alpha_us = k.alpha * 1e6;
  p->link_gbps = k.link / 1e9;
  p->hbm_gbps = k.hbm / 1e9;
  p->issue_us = k.issue * 1e6;
  p->barrier_us = k.barrier * 1e6;
  p->peer_read_gbps = k.peer_read / 1e9;
  p->peer_write_gbps = k.peer_write / 1e9;
  p->copy_gbps = k.copy / 1e9;
  p->coll_gbps = k.coll / 1e9;
  return FTAR_SUCCESS;
}

// the three constants of the round-2 API (kept: bench.py and the C5 line item use them)
ftar_status_t ftar_cost_set_params(double alpha_us, double link_gbps, double hbm_gbps) {
  std::lock_guard<std::mutex> g(ftar::g_cost_mu);
  ftar::g_set.alpha_us = alpha_us > 0 ? alpha_us : 0;
  ftar::g_set.link_gbps = link_gbps > 0 ? link_gbps : 0;
  ftar::g_set.hbm_gbps = hbm_gbps > 0 ? hbm_gbps : 0;
  ++ftar::g_generation;
  return FTAR_SUCCESS;
}

ftar_status_t ftar_cost_get_params(double* alpha_us, double* link_gbps, double* hbm_gbps) {
  const ftar::CostParams k = ftar::cost_params();
  if (alpha_us) *alpha_us = k.alpha * 1e6;
  if (link_gbps) *link_gbps = k.link / 1e9;
  if (hbm_gbps) *hbm_gbps = k.hbm / 1e9;
  return FTAR_SUCCESS;
}

double ftar_cost_predict(const ftar_topo_t* topo, int form, size_t chunk_bytes, int nranks, size_t bytes,
                         int registered) {
  ftar::Topology t;
  if (!topo || ftar::to_topology(topo, nranks, &t) != FTAR_SUCCESS) return -1.0;
  return ftar::exec_cost(t, nranks, bytes, form, chunk_bytes, registered != 0, ftar::cost_params());
}

ftar_status_t ftar_exec_choose(int nranks, size_t bytes, int flags, ftar_exec_t* inout) {
  if (!inout || nranks <= 0) return FTAR_ERR_INVALID_ARG;
  ftar::Topology fixed;
  if (!(flags & FTAR_CHOOSE_TOPO)) FTAR_RETURN_IF(ftar::to_topology(&inout->topo, nranks, &fixed));
  ftar::ExecChoice ch;
  FTAR_RETURN_IF(ftar::choose_exec(nranks, bytes, flags, fixed, inout->form, inout->chunk_bytes, &ch));
  ftar::from_topology(ch.topo, &inout->topo);
  inout->form = ch.form;
  inout->chunk_bytes = ch.chunk;
  inout->seconds = ch.seconds;
  inout->tied = ch.tied;
  inout->tie_broken_by = ch.tie_broken_by;
  return FTAR_SUCCESS;
}

// Topology only (the reference's question, CostModel.h:82-120), at the default data movement: the model's
// best (topology, piece) under the one-round direct forms.  FTAR_COST_MODEL=reference: the reference's own
// scores (capi.cpp).
ftar_status_t ftar_topo_choose(int nranks, size_t bytes, ftar_topo_t* out) {
  if (!out || nranks <= 0) return FTAR_ERR_INVALID_ARG;
  if (const char* m = getenv("FTAR_COST_MODEL")) {
    if (!strcmp(m, "reference")) {  // the reference's own scores (CostModel.h), chunk = FTAR_COST_REF_CHUNK
      const char* ch = getenv("FTAR_COST_REF_CHUNK");
      return ftar_topo_choose_reference(nranks, ch ? atof(ch) : 100.0, out, nullptr);
    }
    if (*m && strcmp(m, "xgmi")) {
      ftar::set_error(std::string("FTAR_COST_MODEL=") + m + ": expected xgmi or reference", __FILE__, __LINE__);
      return FTAR_ERR_INVALID_ARG;
    }
  }
  ftar::Topology ring;
  ring.ring = true;
  ring.widths = {1};
  if (nranks <= 1) {
    ftar::from_topology(ring, out);
    return FTAR_SUCCESS;
  }
  ftar::ExecChoice ch;
  FTAR_RETURN_IF(ftar::choose_exec(nranks, bytes, FTAR_CHOOSE_TOPO | FTAR_CHOOSE_CHUNK, ring, FTAR_FORM_DIRECT, 0,
                                   &ch));
  ftar::from_topology(ch.topo, out);
  return FTAR_SUCCESS;
}

// Model cost (seconds) of one topology at the default data movement (one-round direct forms) and its best
// piece size.
double ftar_topo_cost(const ftar_topo_t* topo, int nranks, size_t bytes) {
  ftar::Topology t;
  if (!topo || ftar::to_topology(topo, nranks, &t) != FTAR_SUCCESS) return -1.0;
  ftar::ExecChoice ch;
  if (ftar::choose_exec(nranks, bytes, FTAR_CHOOSE_CHUNK, t, FTAR_FORM_DIRECT, 0, &ch) != FTAR_SUCCESS) return -1.0;
  return ch.seconds;
}

}  // extern "C"
