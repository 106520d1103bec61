// FlexTree schedule -> executable per-rank plan.
//
// Semantics follow the reference exactly (the tests compare the FMA-level
// schedule with tests/golden/schedules.jsonl, dumped from the reference, and
// the end results with its golden vectors):
//   topology parsing        mpi_mod.hpp:1419-1486  (get_stages)
//   block split             mpi_mod.hpp:776-798, :520-550 (ceil(count/P) per block, P = all ranks)
//   logical send schedule   mpi_mod.hpp:258-347    (Send_Operations, lonely extension :298-345)
//   logical recv schedule   mpi_mod.hpp:349-451    (Recv_Operations, lonely extension :387-449)
//   lonely helpers          mpi_mod.hpp:207-255
//   range lowering          mpi_mod.hpp:627-766    (FMA_Send/Recv_Operations)
//   reduce order            mpi_mod.hpp:1316-1358  (own block first, then peers in op order)
//   ring                    mpi_mod.hpp:1673-1719
// What differs (performance only, never values):
//   * scratch layout is compact (each received range gets its own slot, the
//     self-slot and the reference's 2*aligned buffer are gone) and stages
//     alternate two halves so a stage's receives never overwrite partials a
//     previous stage's reduce may still be reading on the other stream;
//   * the plan is built once per (topology, count) and cached by the engine.
#include <cstdio>
#include <sstream>

#include "ftar_internal.h"

namespace ftar {

std::string Topology::key() const {
  if (ring) return "ring";
  std::string s;
  for (size_t i = 0; i < widths.size(); ++i) s += (i ? "," : "") + std::to_string(widths[i]);
  if (lonely) s += "+" + std::to_string(lonely);
  return s;
}

ftar_status_t to_topology(const ftar_topo_t* t, int nranks, Topology* out) {
  if (!t || !out || nranks <= 0) return FTAR_ERR_INVALID_ARG;
  Topology r;
  if (t->ring) {
    r.ring = true;
    r.widths = {1};
    *out = r;
    return FTAR_SUCCESS;
  }
  if (t->nstages <= 0 || t->nstages > FTAR_MAX_STAGES || t->lonely < 0) return FTAR_ERR_INVALID_TOPO;
  size_t prod = 1;
  for (int i = 0; i < t->nstages; ++i) {
    if (t->stages[i] == 1) {  // any width 1 => ring (mpi_mod.hpp:1461-1464)
      r.ring = true;
      r.widths = {1};
      r.lonely = 0;
      *out = r;
      return FTAR_SUCCESS;
    }
    if (t->stages[i] < 1) return FTAR_ERR_INVALID_TOPO;
    r.widths.push_back((size_t)t->stages[i]);
    prod *= (size_t)t->stages[i];
  }
  r.lonely = (size_t)t->lonely;
  // validity (mpi_mod.hpp:1471): prod + lonely == P, lonely needs >= 2 stages,
  // and the lonely scheme maps lonely rank l onto rank (l * w0) (mpi_mod.hpp:324).
  if (prod + r.lonely != (size_t)nranks) return FTAR_ERR_INVALID_TOPO;
  if (r.lonely && (r.widths.size() < 2 || r.lonely * r.widths[0] > prod)) return FTAR_ERR_INVALID_TOPO;
  *out = r;
  return FTAR_SUCCESS;
}

void from_topology(const Topology& t, ftar_topo_t* out) {
  *out = ftar_topo_t{};
  if (t.ring) {
    out->ring = 1;
    out->nstages = 1;
    out->stages[0] = 1;
    return;
  }
  out->nstages = (int)t.widths.size();
  for (size_t i = 0; i < t.widths.size(); ++i) out->stages[i] = (int)t.widths[i];
  out->lonely = (int)t.lonely;
}

namespace {

// One logical transfer: a peer and the block ids exchanged with it.
struct Peer {
  size_t peer;
  std::vector<size_t> blocks;
};
using PeerList = std::vector<Peer>;

// The FlexTree mixed-radix structure for one rank.
class Tree {
 public:
  Tree(const Topology& t, size_t P, size_t me) : w_(t.widths), P_(P), L_(t.lonely), S_(P - t.lonely), me_(me) {}

  size_t stages() const { return w_.size(); }
  bool lonely_rank() const { return me_ >= S_; }

  // Send_Operations::generate / Recv_Operations::generate, per stage.
  // false where the reference would assert (followers > 1, mpi_mod.hpp:281, :366, :444)
  bool build(std::vector<PeerList>* send, std::vector<PeerList>* send_l, std::vector<PeerList>* recv,
             std::vector<PeerList>* recv_l) const {
    bool ok = true;
    if (!lonely_rank()) {
      for (size_t i = 0, g = 1; i < stages(); g *= w_[i], ++i) {
        const size_t G = g * w_[i];
        const size_t first = me_ / G * G + me_ % g;  // smallest rank of my stage-i group
        const std::vector<size_t> mine = residues(me_, G);
        const auto my_followers = followers(i + 1, me_);
        if (my_followers.size() > 1) ok = false;
        PeerList s, sl, r, rl;
        for (size_t j = 0; j < w_[i]; ++j) {
          const size_t p = first + j * g;
          s.push_back({p, residues(p, G)});
          r.push_back({p, mine});
          if (owns_lonely(i, me_)) {
            auto f = followers(i + 1, p);
            if (f.size() > 1) ok = false;
            if (f.size() == 1) sl.push_back(i + 1 < stages() ? Peer{p, {f[0]}} : Peer{f[0], {f[0]}});
          }
          if (!my_followers.empty() && owns_lonely(i, p) && i + 1 < stages()) rl.push_back({p, {my_followers[0]}});
        }
        if (i == 0 && L_ > 0 && me_ < w_[0] * L_) {  // extended first-stage group (mpi_mod.hpp:298-312)
          const size_t lonely_peer = S_ + me_ / w_[0];
          s.push_back({lonely_peer, lonely_blocks()});
          r.push_back({lonely_peer, mine});
        }
        send->push_back(s);
        send_l->push_back(sl);
        recv->push_back(r);
        recv_l->push_back(rl);
      }
    } else {
      // a lonely rank (mpi_mod.hpp:318-345 and :403-449)
      const size_t base = (me_ - S_) * w_[0];
      PeerList s0, s1, r0, r1;
      for (size_t i = 0; i < w_[0]; ++i) {
        s0.push_back({base + i, residues(base + i, w_[0])});
        r0.push_back({base + i, lonely_blocks()});
      }
      for (size_t b = S_; b < P_; ++b) {
        s1.push_back({b, {b}});
        r1.push_back({b, {me_}});
      }
      send_l->push_back(s0);
      send_l->push_back(s1);
      recv_l->push_back(r0);
      recv_l->push_back(r1);
      for (size_t i = 2; i < stages(); ++i) {
        send_l->emplace_back();
        recv_l->emplace_back();
      }
      PeerList& last = recv_l->back();
      const long step = (long)(S_ / w_.back());
      for (long i = (long)me_ - (long)w_[0]; i >= 0; i -= step) {
        auto f = followers(stages() - 1, (size_t)i);
        if (f.size() == 1 && f[0] != me_) ok = false;
        if (f.size() == 1) last.push_back({(size_t)i, {me_}});
      }
    }
    return ok;
  }

 private:
  // block ids b < S with b ≡ p (mod G)  (Operation(peer, total, gap), mpi_mod.hpp:105-112)
  std::vector<size_t> residues(size_t p, size_t G) const {
    std::vector<size_t> v;
    for (size_t b = p % G; b < S_; b += G) v.push_back(b);
    return v;
  }
  std::vector<size_t> lonely_blocks() const {
    std::vector<size_t> v;
    for (size_t b = S_; b < P_; ++b) v.push_back(b);
    return v;
  }
  size_t gap(size_t h) const {
    size_t g = 1;
    for (size_t i = 0; i < h && i < w_.size(); ++i) g *= w_[i];
    return g;
  }
  // mpi_mod.hpp:207-218
  bool owns_lonely(size_t h, size_t n) const {
    return L_ > 0 && n >= w_[0] * L_ && (h == 0 || n % w_[0] < L_);
  }
  // lonely blocks travelling with rank n at height h (mpi_mod.hpp:224-255)
  std::vector<size_t> followers(size_t h, size_t n) const {
    if (L_ == 0 || !owns_lonely(h, n)) return {};
    const size_t g = gap(h);
    std::vector<size_t> f;
    for (size_t b = S_; b < P_; ++b)
      if ((b - w_[0]) % g == n % g) f.push_back(b);
    return f;
  }

  std::vector<size_t> w_;
  size_t P_, L_, S_, me_;
};

struct Range {
  size_t addr, len, actual;
};
struct MemOp {
  size_t peer;
  bool from_src;
  std::vector<Range> r;
};
using MemStage = std::vector<MemOp>;

struct Fma {
  std::vector<MemStage> send, send_l, recv, recv_l;  // 2k stages (those that exist)
};

Range block_range(size_t b, size_t P, size_t count) {
  const size_t split = (count + P - 1) / P;
  const size_t actual = split * b;
  size_t len = 0;
  if (actual <= count) len = actual + split > count ? count - actual : split;
  return {actual, len, actual};
}

// FMA lowering (mpi_mod.hpp:635-689, :699-765)
Fma lower(const Topology& t, size_t P, size_t me, size_t count, bool* ok = nullptr) {
  std::vector<PeerList> S, SL, R, RL;
  const bool good = Tree(t, P, me).build(&S, &SL, &R, &RL);
  if (ok) *ok = good;
  const size_t k = t.widths.size();
  const size_t split = (count + P - 1) / P;
  auto as_sends = [&](const PeerList& pl, bool from_src) {
    MemStage ms;
    for (auto& p : pl) {
      MemOp m{p.peer, from_src, {}};
      for (size_t b : p.blocks) m.r.push_back(block_range(b, P, count));
      ms.push_back(m);
    }
    return ms;
  };
  auto as_recvs = [&](const PeerList& pl, bool at_block, size_t tile) {
    MemStage ms;
    for (auto& p : pl) {
      MemOp m{p.peer, false, {}};
      for (size_t b : p.blocks) {
        Range r = block_range(b, P, count);
        if (!at_block) {
          r.addr = tile;
          tile += split;
        }
        m.r.push_back(r);
      }
      ms.push_back(m);
    }
    return ms;
  };
  Fma f;
  for (size_t i = 0; i < S.size(); ++i) f.send.push_back(as_sends(S[i], i == 0));
  for (size_t i = R.size(); i-- > 0;) f.send.push_back(as_sends(R[i], false));
  for (size_t i = 0; i < SL.size(); ++i) f.send_l.push_back(as_sends(SL[i], i == 0));
  for (size_t i = RL.size(); i-- > 0;) f.send_l.push_back(as_sends(RL[i], false));
  for (size_t i = 0; i < R.size(); ++i) f.recv.push_back(as_recvs(R[i], false, 0));
  for (size_t i = S.size(); i-- > 0;) f.recv.push_back(as_recvs(S[i], true, 0));
  for (size_t i = 0; i < RL.size(); ++i) f.recv_l.push_back(as_recvs(RL[i], false, split * P));
  for (size_t i = SL.size(); i-- > 0;) f.recv_l.push_back(as_recvs(SL[i], true, 0));
  (void)k;
  return f;
}

void json_stages(std::ostringstream& os, const std::vector<MemStage>& v) {
  os << "[";
  for (size_t i = 0; i < v.size(); ++i) {
    os << (i ? "," : "") << "[";
    for (size_t j = 0; j < v[i].size(); ++j) {
      const MemOp& m = v[i][j];
      os << (j ? "," : "") << "{\"peer\":" << m.peer << ",\"src\":" << (m.from_src ? 1 : 0) << ",\"r\":[";
      for (size_t q = 0; q < m.r.size(); ++q)
        os << (q ? "," : "") << "[" << m.r[q].addr << "," << m.r[q].len << "," << m.r[q].actual << "]";
      os << "]}";
    }
    os << "]";
  }
  os << "]";
}

// Build one reduce-scatter stage of the tree plan from the FMA ops of stage i.
void add_tree_stage(Stage& st, size_t me, const MemStage* send, const MemStage* send_l, const MemStage* recv,
                    const MemStage* recv_l, bool first, size_t scratch_base, size_t* scratch_used, int* max_k) {
  auto emit_sends = [&](const MemStage* ms) {
    if (!ms || ms->empty()) return;
    const int buf = (*ms)[0].from_src ? BUF_SRC : BUF_DST;  // mpi_mod.hpp:1559 (first op decides)
    for (auto& m : *ms)
      if (m.peer != me)
        for (auto& r : m.r)
          if (r.len) st.sends.push_back({(int)m.peer, buf, r.addr, r.len});
  };
  emit_sends(send);
  emit_sends(send_l);
  // receive into compact scratch slots; remember each (op, range) slot for the reduce
  auto emit_recvs = [&](const MemStage* ms, std::vector<std::vector<size_t>>* slot) {
    if (!ms) return;
    for (auto& m : *ms) {
      slot->emplace_back(m.r.size(), (size_t)-1);
      if (m.peer == me) continue;
      for (size_t q = 0; q < m.r.size(); ++q) {
        if (!m.r[q].len) continue;
        const size_t off = scratch_base + *scratch_used;
        *scratch_used += m.r[q].len;
        st.recvs.push_back({(int)m.peer, BUF_SCRATCH, off, m.r[q].len});
        slot->back()[q] = off;
      }
    }
  };
  std::vector<std::vector<size_t>> slot_main, slot_l;
  emit_recvs(recv, &slot_main);
  emit_recvs(recv_l, &slot_l);
  // handle_reduce (mpi_mod.hpp:1316-1358): per block index, own block + peers in op order;
  // k <= 1 is a no-op (mpi_mod.hpp:819)
  auto emit_reduces = [&](const MemStage* ms, const std::vector<std::vector<size_t>>& slot) {
    if (!ms || ms->empty()) return;
    const MemOp& lead = (*ms)[0];
    for (size_t q = 0; q < lead.r.size(); ++q) {
      if (!lead.r[q].len) continue;
      ReduceItem it{lead.r[q].actual, lead.r[q].len, {{first ? BUF_SRC : BUF_DST, lead.r[q].actual}}};
      for (size_t j = 0; j < ms->size(); ++j)
        if ((*ms)[j].peer != me) it.srcs.push_back({BUF_SCRATCH, slot[j][q]});
      if (it.srcs.size() < 2) continue;
      *max_k = std::max(*max_k, (int)it.srcs.size());
      st.reduces.push_back(std::move(it));
    }
  };
  emit_reduces(recv, slot_main);
  emit_reduces(recv_l, slot_l);
}

}  // namespace

ftar_status_t schedule_json(const Topology& t, int nranks, int rank, size_t count, std::string* out) {
  if (t.ring || rank < 0 || rank >= nranks) return FTAR_ERR_INVALID_ARG;
  Fma f = lower(t, (size_t)nranks, (size_t)rank, count);
  std::ostringstream os;
  os << "{\"send\":";
  json_stages(os, f.send);
  os << ",\"send_lonely\":";
  json_stages(os, f.send_l);
  os << ",\"recv\":";
  json_stages(os, f.recv);
  os << ",\"recv_lonely\":";
  json_stages(os, f.recv_l);
  os << "}";
  *out = os.str();
  return FTAR_SUCCESS;
}

namespace {
// One-round all-gather: after the reduce-scatter stages rank q holds the final
// value of exactly one block, owner_block(q); send mine to every peer, receive
// each peer's (ascending peer order on both sides, so per-pair FIFO matches).
Stage direct_allgather_stage(size_t P, size_t me, size_t count, bool ring) {
  auto owner_block = [&](size_t q) { return ring ? (q + 1) % P : q; };
  Stage st;
  const Range mine = block_range(owner_block(me), P, count);
  for (size_t p = 0; p < P; ++p) {
    if (p == me) continue;
    if (mine.len) st.sends.push_back({(int)p, BUF_DST, mine.actual, mine.len});
    const Range theirs = block_range(owner_block(p), P, count);
    if (theirs.len) st.recvs.push_back({(int)p, BUF_DST, theirs.actual, theirs.len});
  }
  return st;
}
// Depth-first leaf order of block n's fold tree after s stages: the stage-s
// reduce at rank n folds its own partial, then its stage group's partials in
// ascending rank order (mpi_mod.hpp:1316-1358); every partial is itself the
// fold of the previous stage's group.  Rank n's group at stage s is
// {left + j*g : j < w_s}, g = w_0...w_{s-1}, left = n's window start + n mod g
// (mpi_mod.hpp:80-140).
void tree_leaves(const std::vector<size_t>& w, size_t n, size_t s, std::vector<size_t>* out) {
  if (s == 0) {
    out->push_back(n);
    return;
  }
  tree_leaves(w, n, s - 1, out);
  size_t g = 1;
  for (size_t i = 0; i + 1 < s; ++i) g *= w[i];
  const size_t G = g * w[s - 1], left = n / G * G + n % g;
  for (size_t j = 0; j < w[s - 1]; ++j)
    if (left + j * g != n) tree_leaves(w, left + j * g, s - 1, out);
}

// One-round reduce-scatter of a multi-stage tree without lonely ranks: every
// rank sends its copy of block q to rank q and folds the P copies of its own
// block in one nested k = P fold (leaves in tree_leaves order, shape = the
// stage widths): the staged tree's values, bit for bit, with all links busy
// at once instead of one stage group at a time.
Stage direct_tree_stage(const Topology& t, size_t P, size_t me, size_t count) {
  Stage st;
  for (size_t q = 0; q < P; ++q) {
    if (q == me) continue;
    const Range c = block_range(q, P, count);
    if (c.len) st.sends.push_back({(int)q, BUF_SRC, c.actual, c.len});
  }
  const Range mine = block_range(me, P, count);
  if (!mine.len) return st;
  std::vector<size_t> leaves;
  tree_leaves(t.widths, me, t.widths.size(), &leaves);
  ReduceItem it{mine.actual, mine.len, {}, false, {}};
  for (size_t w : t.widths) it.shape.push_back((int)w);
  size_t slot = 0;
  for (size_t q : leaves) {
    if (q == me) {
      it.srcs.push_back({BUF_SRC, mine.actual});
      continue;
    }
    st.recvs.push_back({(int)q, BUF_SCRATCH, slot, mine.len});
    it.srcs.push_back({BUF_SCRATCH, slot});
    slot += mine.len;
  }
  st.reduces.push_back(std::move(it));
  return st;
}
}  // namespace

ftar_status_t build_plan(const Topology& t, int nranks, int rank, size_t count, Plan* out, Form form) {
  const int allgather = form.allgather;
  if (rank < 0 || rank >= nranks) return FTAR_ERR_INVALID_ARG;
  Plan p;
  p.rank = rank;
  p.nranks = nranks;
  p.count = count;
  const size_t P = (size_t)nranks, me = (size_t)rank;
  p.split = (count + P - 1) / P;
  if (nranks == 1) {
    *out = p;
    return FTAR_SUCCESS;
  }
  size_t half = 0;
  if (t.ring) {
    // ring_allreduce (mpi_mod.hpp:1673-1719): step i sends block (me-i) to the
    // right neighbour and folds block (me-1-i) from the left into it:
    // dst = own(sendbuf) + recv, own always from the caller's send buffer.
    const int right = (int)((me + 1) % P), left = (int)((me + P - 1) % P);
    size_t bs = me, br = (me + P - 1) % P;
    if (form.reduce_scatter == FTAR_RS_DIRECT && P <= FTAR_MAX_K) {  // one k = P fold
      // one round: block b = (me+1) mod P is folded here from every rank's copy,
      // in the ring's order b, b+1, ..., b+P-1 (= me, the caller's own copy last)
      Stage st;
      const size_t ob = (me + 1) % P;
      for (size_t q = 0; q < P; ++q) {  // my copy of the block rank q owns
        if (q == me) continue;
        const Range c = block_range((q + 1) % P, P, count);
        if (c.len) st.sends.push_back({(int)q, BUF_SRC, c.actual, c.len});
      }
      const Range mine = block_range(ob, P, count);
      if (mine.len) {
        ReduceItem it{mine.actual, mine.len, {}, true};
        size_t slot = 0;
        for (size_t j = 0; j < P; ++j) {
          const size_t q = (ob + j) % P;
          if (q == me) {
            it.srcs.push_back({BUF_SRC, mine.actual});
            continue;
          }
          st.recvs.push_back({(int)q, BUF_SCRATCH, slot, mine.len});
          it.srcs.push_back({BUF_SCRATCH, slot});
          slot += mine.len;
        }
        st.reduces.push_back(std::move(it));
      }
      p.stages.push_back(std::move(st));
      p.reduce_scatter = FTAR_RS_DIRECT;
      half = (P - 1) * p.split;
      p.max_k = (int)P;
      bs = (me + 1) % P;  // where the staged loop would leave them
      br = me;
    } else {
      for (size_t i = 0; i + 1 < P; ++i) {
        Stage st;
        Range s = block_range(bs, P, count), r = block_range(br, P, count);
        if (s.len) st.sends.push_back({right, i == 0 ? BUF_SRC : BUF_DST, s.actual, s.len});
        const size_t base = (i % 2) * p.split;
        if (r.len) {
          st.recvs.push_back({left, BUF_SCRATCH, base, r.len});
          st.reduces.push_back({r.actual, r.len, {{BUF_SRC, r.actual}, {BUF_SCRATCH, base}}, true});
        }
        p.stages.push_back(std::move(st));
        bs = (bs + P - 1) % P;
        br = (br + P - 1) % P;
      }
      half = p.split;
      p.max_k = 2;
    }
    if (allgather == FTAR_AG_STAGES) {
      for (size_t i = 0; i + 1 < P; ++i) {  // mpi_mod.hpp:1705-1715
        Stage st;
        Range s = block_range(bs, P, count), r = block_range(br, P, count);
        if (s.len) st.sends.push_back({right, BUF_DST, s.actual, s.len});
        if (r.len) st.recvs.push_back({left, BUF_DST, r.actual, r.len});
        p.stages.push_back(std::move(st));
        bs = (bs + P - 1) % P;
        br = (br + P - 1) % P;
      }
      p.allgather = FTAR_AG_STAGES;
    } else {  // the ring's final blocks sit one rank off: no collective layout, go direct
      p.stages.push_back(direct_allgather_stage(P, me, count, true));
      p.allgather = FTAR_AG_DIRECT;
    }
  } else {
    bool good = true;
    Fma f = lower(t, P, me, count, &good);
    if (!good) return FTAR_ERR_INVALID_TOPO;
    const size_t k = t.widths.size();
    auto at = [](const std::vector<MemStage>& v, size_t i) -> const MemStage* { return i < v.size() ? &v[i] : nullptr; };
    int max_k = 0;
    const bool direct_rs = form.reduce_scatter == FTAR_RS_DIRECT && t.lonely == 0 && k >= 2 &&
                           k <= (size_t)kMaxFoldLevels && P <= FTAR_MAX_K;
    if (direct_rs) {
      p.stages.push_back(direct_tree_stage(t, P, me, count));
      p.reduce_scatter = FTAR_RS_DIRECT;
      half = (P - 1) * p.split;
      max_k = (int)P;
    }
    // pass 1: scratch needed per reduce-scatter stage
    std::vector<Stage> rs(k);
    std::vector<size_t> used(k, 0);
    for (size_t i = 0; i < k && !direct_rs; ++i) {
      add_tree_stage(rs[i], me, at(f.send, i), at(f.send_l, i), at(f.recv, i), at(f.recv_l, i), i == 0, 0, &used[i],
                     &max_k);
      half = std::max(half, used[i]);
    }
    // pass 2: rebuild with each stage in its half (stages alternate halves)
    for (size_t i = 0; i < k && !direct_rs; ++i) {
      Stage st;
      size_t u = 0;
      add_tree_stage(st, me, at(f.send, i), at(f.send_l, i), at(f.recv, i), at(f.recv_l, i), i == 0, (i % 2) * half,
                     &u, &max_k);
      p.stages.push_back(std::move(st));
    }
    // all-gather: the reference's reversed stages straight into dst (mpi_mod.hpp:1620-1644),
    // one direct round, or one collective
    if (allgather == FTAR_AG_COLLECTIVE && t.lonely == 0 && count % P == 0) p.allgather = FTAR_AG_COLLECTIVE;
    else if (allgather == FTAR_AG_STAGES) p.allgather = FTAR_AG_STAGES;
    else {
      p.allgather = FTAR_AG_DIRECT;
      p.stages.push_back(direct_allgather_stage(P, me, count, false));
    }
    for (size_t i = k; i < 2 * k && p.allgather == FTAR_AG_STAGES; ++i) {
      Stage st;
      for (const MemStage* ms : {at(f.send, i), at(f.send_l, i)})
        if (ms)
          for (auto& m : *ms)
            if (m.peer != me)
              for (auto& r : m.r)
                if (r.len) st.sends.push_back({(int)m.peer, BUF_DST, r.addr, r.len});
      for (const MemStage* ms : {at(f.recv, i), at(f.recv_l, i)})
        if (ms)
          for (auto& m : *ms)
            if (m.peer != me)
              for (auto& r : m.r)
                if (r.len) st.recvs.push_back({(int)m.peer, BUF_DST, r.addr, r.len});
      p.stages.push_back(std::move(st));
    }
    p.max_k = max_k;
  }
  p.scratch_half = half;
  *out = std::move(p);
  return FTAR_SUCCESS;
}

// Every rank's plan, built here, must pair up: per stage and per (sender,
// receiver), the sender's transfers to the receiver and the receiver's
// transfers from the sender have the same lengths in the same order (RCCL and
// MPI match p2p messages per peer pair in posting order).  Topologies the
// reference cannot run (its asserts, or schedules that would block in
// MPI_Waitall) fail here instead of hanging a collective.
ftar_status_t check_world(const Topology& t, int nranks, size_t count, Form form) {
  std::vector<Plan> plans(nranks);
  for (int r = 0; r < nranks; ++r) FTAR_RETURN_IF(build_plan(t, nranks, r, count, &plans[r], form));
  for (int r = 1; r < nranks; ++r)
    if (plans[r].stages.size() != plans[0].stages.size()) return FTAR_ERR_INVALID_TOPO;
  for (size_t s = 0; s < plans[0].stages.size(); ++s)
    for (int a = 0; a < nranks; ++a)
      for (int b = 0; b < nranks; ++b) {
        if (a == b) continue;
        std::vector<size_t> sent, got;
        for (const Transfer& x : plans[a].stages[s].sends)
          if (x.peer == b) sent.push_back(x.len);
        for (const Transfer& x : plans[b].stages[s].recvs)
          if (x.peer == a) got.push_back(x.len);
        if (sent != got) return FTAR_ERR_INVALID_TOPO;
      }
  return FTAR_SUCCESS;
}

std::string Plan::json() const {
  std::ostringstream os;
  static const char* bn[] = {"src", "dst", "scratch"};
  os << "{\"rank\":" << rank << ",\"nranks\":" << nranks << ",\"count\":" << count << ",\"split\":" << split
     << ",\"scratch_half\":" << scratch_half << ",\"max_k\":" << max_k
     << ",\"allgather\":\"" << (allgather == FTAR_AG_COLLECTIVE ? "collective" : allgather == FTAR_AG_DIRECT ? "direct" : "stages")
     << "\",\"reduce_scatter\":\"" << (reduce_scatter == FTAR_RS_DIRECT ? "direct" : "stages") << "\",\"stages\":[";
  for (size_t i = 0; i < stages.size(); ++i) {
    const Stage& s = stages[i];
    os << (i ? "," : "") << "{\"sends\":[";
    for (size_t j = 0; j < s.sends.size(); ++j)
      os << (j ? "," : "") << "[" << s.sends[j].peer << ",\"" << bn[s.sends[j].buf] << "\"," << s.sends[j].off << ","
         << s.sends[j].len << "]";
    os << "],\"recvs\":[";
    for (size_t j = 0; j < s.recvs.size(); ++j)
      os << (j ? "," : "") << "[" << s.recvs[j].peer << ",\"" << bn[s.recvs[j].buf] << "\"," << s.recvs[j].off << ","
         << s.recvs[j].len << "]";
    os << "],\"reduces\":[";
    for (size_t j = 0; j < s.reduces.size(); ++j) {
      const ReduceItem& r = s.reduces[j];
      os << (j ? "," : "") << "{\"off\":" << r.off << ",\"len\":" << r.len << ",\"round_each\":"
         << (r.round_each ? 1 : 0) << ",\"shape\":[";
      for (size_t q = 0; q < r.shape.size(); ++q) os << (q ? "," : "") << r.shape[q];
      os << "],\"srcs\":[";
      for (size_t q = 0; q < r.srcs.size(); ++q)
        os << (q ? "," : "") << "[\"" << bn[r.srcs[q].buf] << "\"," << r.srcs[q].off << "]";
      os << "]}";
    }
    os << "]}";
  }
  os << "]}";
  return os.str();
}

}  // namespace ftar
