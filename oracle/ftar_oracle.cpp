// ============================================================================
// ftar ORACLE — TEST INFRASTRUCTURE ONLY.
//
// A CPU restatement of the reference FlexTree AllReduce
// (/root/reference/allreduce_over_mpi/mpi_mod.hpp) used as the *checker* for
// the MI355X product in allreduce-over-mpi_amd/.  Only tests/, the smoke()
// entry of __graft_entry__.py and bench.py's cpu_baseline leg may load this
// library.  The product never links, loads or falls back to it.
//
// Parity of this oracle is pinned against golden vectors produced by the
// reference itself (oracle/ref_golden.cpp compiled against the unmodified
// reference header under MPICH, see oracle/Makefile and oracle/gen_golden.py);
// tests/test_oracle_golden.py checks every committed fixture bit-for-bit.
//
// What is restated (reference file:line):
//   reduce_sum<T>        mpi_mod.hpp:811-1031   left-to-right k-way sum, k<=1 no-op
//   reduce_band<T>       mpi_mod.hpp:1033-1251  k-way bitwise AND
//   reduce_sum (copy k1) vector_add/reduce_sum.h:36-47  (kernel-harness variant)
//   Send_Operations      mpi_mod.hpp:258-347    logical send schedule incl. lonely
//   Recv_Operations      mpi_mod.hpp:349-451    logical recv schedule incl. lonely
//   Operations helpers   mpi_mod.hpp:207-255    has_lonely_blocks/find_star/find_followers
//   FMA_* lowering       mpi_mod.hpp:459-766    blocks -> element ranges, recv tiling
//   tree_allreduce       mpi_mod.hpp:1510-1671  stage loop, reduce order
//   ring_allreduce       mpi_mod.hpp:1673-1719  2(P-1) steps, own+recv order
//   MPI_Allreduce_FT     mpi_mod.hpp:1723-1778  dispatch, P<=1 memcpy
// Transport (MPI_Isend/Irecv, tag 0, per-pair FIFO matching) is simulated in
// memory, all P ranks in one process, one stage at a time.
//
// bf16 is NOT in the reference (mpi_mod.hpp:1365-1375 has no 16-bit float);
// its semantics here are this project's definition (fp32 accumulate per
// reduce call, one round-to-nearest-even per call) and are parity-UNPINNED.
// ============================================================================
#include <cstdint>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>
#include <deque>
#include <map>
#include <sstream>
#include <stdexcept>

namespace oracle {

enum Dtype { U8 = 0, I8, U16, I16, I32, I64, F32, F64, BOOL, BF16, NDTYPE };
enum Op { SUM = 0, BAND = 1 };

static size_t dtype_size(int dt) {
  static const size_t sz[] = {1, 1, 2, 2, 4, 8, 4, 8, 1, 2};
  if (dt < 0 || dt >= NDTYPE) throw std::runtime_error("bad dtype");
  return sz[dt];
}

// --------------------------------------------------------------------------
// element-wise reduce (mpi_mod.hpp:812-1031, :1034-1251)
// --------------------------------------------------------------------------
static inline float bf16_to_f32(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
static inline uint16_t f32_to_bf16_rne(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // NaN stays NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

template <class T>
static void sum_loop(const void* const* src, void* dst, int k, size_t n) {
  // C++ semantics of `dst[i] = src0[i] + src1[i] + ...`: operands promote to
  // int for the narrow integer types and to nothing for float/double, are
  // added strictly left to right, and the result converts back to T on the
  // store (modular for integers, `!= 0` for bool).
  const T* const* s = reinterpret_cast<const T* const*>(src);
  T* d = static_cast<T*>(dst);
  for (size_t i = 0; i < n; ++i) {
    T acc = s[0][i];
    for (int j = 1; j < k; ++j) acc = (T)(acc + s[j][i]);
    d[i] = acc;
  }
}
template <class U>  // integers: wrap-around in the unsigned twin (same bits as gcc's code)
static void sum_loop_int(const void* const* src, void* dst, int k, size_t n) {
  const U* const* s = reinterpret_cast<const U* const*>(src);
  U* d = static_cast<U*>(dst);
  for (size_t i = 0; i < n; ++i) {
    U acc = s[0][i];
    for (int j = 1; j < k; ++j) acc = (U)(acc + s[j][i]);
    d[i] = acc;
  }
}
static void sum_loop_bool(const void* const* src, void* dst, int k, size_t n) {
  const uint8_t* const* s = reinterpret_cast<const uint8_t* const*>(src);
  uint8_t* d = static_cast<uint8_t*>(dst);
  for (size_t i = 0; i < n; ++i) {
    int acc = s[0][i] ? 1 : 0;  // bool operands promote to int 0/1
    for (int j = 1; j < k; ++j) acc += s[j][i] ? 1 : 0;
    d[i] = acc != 0;
  }
}
static void sum_loop_bf16(const void* const* src, void* dst, int k, size_t n) {
  const uint16_t* const* s = reinterpret_cast<const uint16_t* const*>(src);
  uint16_t* d = static_cast<uint16_t*>(dst);
  for (size_t i = 0; i < n; ++i) {
    float acc = bf16_to_f32(s[0][i]);
    for (int j = 1; j < k; ++j) acc = acc + bf16_to_f32(s[j][i]);
    d[i] = f32_to_bf16_rne(acc);
  }
}
template <class U>
static void band_loop(const void* const* src, void* dst, int k, size_t n) {
  const U* const* s = reinterpret_cast<const U* const*>(src);
  U* d = static_cast<U*>(dst);
  for (size_t i = 0; i < n; ++i) {
    U acc = s[0][i];
    for (int j = 1; j < k; ++j) acc = (U)(acc & s[j][i]);
    d[i] = acc;
  }
}

// copy_k1: reduce_sum.h (kernel harness) copies for k==1; mpi_mod.hpp:819 does not.
static int reduce(int dt, int op, const void* const* src, int k, void* dst, size_t n, bool copy_k1) {
  if (k <= 0) return 0;
  if (k == 1) {
    if (copy_k1 && dst != src[0]) std::memmove(dst, src[0], n * dtype_size(dt));
    return 0;
  }
  if (op == SUM) {
    switch (dt) {
      case U8: case I8: sum_loop_int<uint8_t>(src, dst, k, n); return 0;
      case U16: case I16: sum_loop_int<uint16_t>(src, dst, k, n); return 0;
      case I32: sum_loop_int<uint32_t>(src, dst, k, n); return 0;
      case I64: sum_loop_int<uint64_t>(src, dst, k, n); return 0;
      case F32: sum_loop<float>(src, dst, k, n); return 0;
      case F64: sum_loop<double>(src, dst, k, n); return 0;
      case BOOL: sum_loop_bool(src, dst, k, n); return 0;
      case BF16: sum_loop_bf16(src, dst, k, n); return 0;
    }
  } else if (op == BAND) {
    switch (dt) {
      case U8: case I8: band_loop<uint8_t>(src, dst, k, n); return 0;
      case U16: case I16: band_loop<uint16_t>(src, dst, k, n); return 0;
      case I32: band_loop<uint32_t>(src, dst, k, n); return 0;
      case I64: band_loop<uint64_t>(src, dst, k, n); return 0;
      default: return -2;  // mpi_mod.hpp:1397-1405: BAND on float/double/bool unsupported
    }
  }
  return -3;
}

// --------------------------------------------------------------------------
// logical schedule (mpi_mod.hpp:80-451)
// --------------------------------------------------------------------------
struct Xfer {
  size_t peer;
  std::vector<size_t> blocks;
};
using StageXfers = std::vector<Xfer>;

struct Topo {
  size_t P, L, S;             // total ranks, lonely ranks, P-L
  std::vector<size_t> w;      // stage widths, bottom-up
  size_t k() const { return w.size(); }
};

// blocks ≡ peer (mod g) below S  (Operation ctor, mpi_mod.hpp:105-112)
static Xfer strided(size_t peer, size_t S, size_t g) {
  Xfer x{peer, {}};
  for (size_t b = peer % g; b < S; b += g) x.blocks.push_back(b);
  return x;
}
static size_t gap_below(const Topo& t, size_t h) {  // prod of widths of stages < h
  size_t g = 1;
  for (size_t i = 0; i < h && i < t.k(); ++i) g *= t.w[i];
  return g;
}
// mpi_mod.hpp:207-218
static bool has_lonely_blocks(const Topo& t, size_t h, size_t n) {
  return t.L > 0 && n >= t.w[0] * t.L && (h == 0 || n % t.w[0] < t.L);
}
// mpi_mod.hpp:224-255 (find_star(b) = b - w0)
static std::vector<size_t> find_followers(const Topo& t, size_t h, size_t n) {
  if (t.L == 0) return {};
  size_t g = gap_below(t, h);
  std::vector<size_t> f;
  for (size_t b = t.S; b < t.P; ++b)
    if ((b - t.w[0]) % g == n % g) f.push_back(b);
  if (!has_lonely_blocks(t, h, n)) return {};
  return f;
}

struct Logical {
  std::vector<StageXfers> main, lonely;  // one entry per stage (k)
};

// Send_Operations::generate, mpi_mod.hpp:263-346
static Logical gen_send(const Topo& t, size_t n) {
  Logical out;
  const size_t k = t.k();
  if (n < t.S) {
    size_t g = 1;
    for (size_t i = 0; i < k; ++i) {
      const size_t G = g * t.w[i];
      StageXfers m, l;
      size_t p = n / G * G + n % g;
      for (size_t j = 0; j < t.w[i]; ++j, p += g) {
        m.push_back(strided(p, t.S, G));
        if (has_lonely_blocks(t, i, n)) {
          auto f = find_followers(t, i + 1, p);
          if (f.size() > 1) throw std::runtime_error("followers > 1");
          if (f.size() == 1) {
            if (i != k - 1) l.push_back({p, {f[0]}});
            else l.push_back({f[0], {f[0]}});
          }
        }
      }
      if (i == 0 && t.L > 0 && n < t.w[0] * t.L) {
        Xfer x{t.S + n / t.w[0], {}};
        for (size_t b = t.S; b < t.P; ++b) x.blocks.push_back(b);
        m.push_back(x);
      }
      out.main.push_back(m);
      out.lonely.push_back(l);
      g = G;
    }
  } else {
    StageXfers s0, s1;
    size_t left = (n - t.S) * t.w[0];
    for (size_t i = 0; i < t.w[0]; ++i) s0.push_back(strided(left + i, t.S, t.w[0]));
    for (size_t b = t.S; b < t.P; ++b) s1.push_back({b, {b}});
    out.lonely.push_back(s0);
    out.lonely.push_back(s1);
    for (size_t i = 2; i < k; ++i) out.lonely.emplace_back();
  }
  return out;
}

// Recv_Operations::generate, mpi_mod.hpp:354-450
static Logical gen_recv(const Topo& t, size_t n) {
  Logical out;
  const size_t k = t.k();
  if (n < t.S) {
    size_t g = 1;
    for (size_t i = 0; i < k; ++i) {
      const size_t G = g * t.w[i];
      StageXfers m, l;
      Xfer mine = strided(n, t.S, G);
      auto f = find_followers(t, i + 1, n);
      if (f.size() > 1) throw std::runtime_error("followers > 1");
      size_t p = n / G * G + n % g;
      for (size_t j = 0; j < t.w[i]; ++j, p += g) {
        Xfer x = mine;
        x.peer = p;
        m.push_back(x);
        if (!f.empty() && has_lonely_blocks(t, i, p) && i != k - 1) l.push_back({p, {f[0]}});
      }
      if (i == 0 && t.L > 0 && n < t.w[0] * t.L) {
        Xfer x = mine;
        x.peer = t.S + n / t.w[0];
        m.push_back(x);
      }
      out.main.push_back(m);
      out.lonely.push_back(l);
      g = G;
    }
  } else {
    StageXfers s0, s1;
    std::vector<size_t> all_lonely;
    for (size_t b = t.S; b < t.P; ++b) all_lonely.push_back(b);
    size_t left = (n - t.S) * t.w[0];
    for (size_t i = 0; i < t.w[0]; ++i) s0.push_back({left + i, all_lonely});
    for (size_t b = t.S; b < t.P; ++b) s1.push_back({b, {n}});
    out.lonely.push_back(s0);
    out.lonely.push_back(s1);
    for (size_t i = 2; i < k; ++i) out.lonely.emplace_back();
    StageXfers& last = out.lonely.back();
    const long g = (long)(t.S / t.w[k - 1]);
    for (long i = (long)n - (long)t.w[0]; i >= 0; i -= g) {
      auto f = find_followers(t, k - 1, (size_t)i);
      if (f.size() == 1) {
        if (f[0] != n) throw std::runtime_error("lonely follower mismatch");
        last.push_back({(size_t)i, {n}});
      }
    }
  }
  return out;
}

// --------------------------------------------------------------------------
// range lowering (FMA_*, mpi_mod.hpp:459-766)
// --------------------------------------------------------------------------
struct Range {
  size_t addr, len, actual;
};
struct MemOp {
  size_t peer;
  bool from_src;
  std::vector<Range> r;
};
using StageMem = std::vector<MemOp>;

// push_block_back, mpi_mod.hpp:520-550 (INF addr == "at the block's own offset")
static Range block_range(size_t b, size_t P, size_t count, size_t addr, bool own_offset) {
  size_t split = (count + P - 1) / P;
  size_t actual = split * b, len;
  if (actual > count) len = 0;
  else if (actual + split > count) len = count - actual;
  else len = split;
  return Range{own_offset ? actual : addr, len, actual};
}

struct RankPlan {
  // 2k stages each; index < k is reduce-scatter, >= k all-gather
  std::vector<StageMem> send_main, send_lonely, recv_main, recv_lonely;
  bool has_main_send = false, has_main_recv = false;
};

static RankPlan lower(const Topo& t, size_t n, size_t count) {
  Logical S = gen_send(t, n), R = gen_recv(t, n);
  const size_t k = t.k(), P = t.P;
  const size_t split = (count + P - 1) / P;
  RankPlan rp;
  auto sends = [&](const StageXfers& xs, bool from_src) {
    StageMem sm;
    for (auto& x : xs) {
      MemOp m{x.peer, from_src, {}};
      for (size_t b : x.blocks) m.r.push_back(block_range(b, P, count, 0, true));
      sm.push_back(m);
    }
    return sm;
  };
  auto recvs = [&](const StageXfers& xs, bool accordingly, size_t offset) {
    StageMem sm;
    for (auto& x : xs) {
      MemOp m{x.peer, false, {}};
      for (size_t b : x.blocks) {
        if (accordingly) m.r.push_back(block_range(b, P, count, 0, true));
        else {
          m.r.push_back(block_range(b, P, count, offset, false));
          offset += split;
        }
      }
      sm.push_back(m);
    }
    return sm;
  };
  // FMA_Send_Operations::generate (mpi_mod.hpp:635-689)
  rp.has_main_send = !S.main.empty();
  rp.has_main_recv = !R.main.empty();
  if (!S.main.empty())
    for (size_t i = 0; i < k; ++i) rp.send_main.push_back(sends(S.main[i], i == 0));
  if (!R.main.empty())
    for (long i = (long)k - 1; i >= 0; --i) rp.send_main.push_back(sends(R.main[i], false));
  if (!S.lonely.empty())
    for (size_t i = 0; i < k; ++i) rp.send_lonely.push_back(sends(S.lonely[i], i == 0));
  if (!R.lonely.empty())
    for (long i = (long)k - 1; i >= 0; --i) rp.send_lonely.push_back(sends(R.lonely[i], false));
  // FMA_Recv_Operations::generate (mpi_mod.hpp:699-765)
  if (!R.main.empty())
    for (size_t i = 0; i < k; ++i) rp.recv_main.push_back(recvs(R.main[i], false, 0));
  if (!S.main.empty())
    for (long i = (long)k - 1; i >= 0; --i) rp.recv_main.push_back(recvs(S.main[i], true, 0));
  const size_t lonely_off = split * P;
  if (!R.lonely.empty())
    for (size_t i = 0; i < k; ++i) rp.recv_lonely.push_back(recvs(R.lonely[i], false, lonely_off));
  if (!S.lonely.empty())
    for (long i = (long)k - 1; i >= 0; --i) rp.recv_lonely.push_back(recvs(S.lonely[i], true, 0));
  return rp;
}

// --------------------------------------------------------------------------
// simulated execution of all P ranks
// --------------------------------------------------------------------------
struct Msg {
  std::vector<uint8_t> bytes;
};

struct World {
  size_t P, count, esz;
  int dt, op;
  std::vector<const uint8_t*> data;  // per-rank send buffer (== dst when in place)
  std::vector<uint8_t*> dst;
  std::vector<std::vector<uint8_t>> scratch;  // recv_buffer (mpi_mod.hpp:1748: 2*aligned)
  std::map<std::pair<size_t, size_t>, std::deque<Msg>> wire;

  void post_send(size_t from, size_t to, const uint8_t* p, size_t len) {
    Msg m;
    m.bytes.assign(p, p + len * esz);
    wire[{from, to}].push_back(std::move(m));
  }
  void complete_recv(size_t from, size_t to, uint8_t* p, size_t len) {
    auto& q = wire[{from, to}];
    if (q.empty()) throw std::runtime_error("recv with no matching send (would deadlock)");
    Msg m = std::move(q.front());
    q.pop_front();
    if (m.bytes.size() != len * esz) throw std::runtime_error("message length mismatch");
    std::memcpy(p, m.bytes.data(), m.bytes.size());
  }
  void check_drained() {
    for (auto& kv : wire)
      if (!kv.second.empty()) throw std::runtime_error("unmatched send left on the wire");
  }
};

// handle_reduce, mpi_mod.hpp:1316-1415
static int do_reduce(World& w, size_t me, const StageMem& ops, const uint8_t* buffer,
                     const uint8_t* own, uint8_t* dest) {
  if (ops.empty()) return 0;
  const size_t nb = ops[0].r.size();
  std::vector<const void*> src;
  for (size_t bi = 0; bi < nb; ++bi) {
    const size_t len = ops[0].r[bi].len;
    if (len == 0) continue;
    src.clear();
    src.push_back(own + ops[0].r[bi].actual * w.esz);
    uint8_t* d = dest + ops[0].r[bi].actual * w.esz;
    for (auto& o : ops)
      if (o.peer != me) src.push_back(buffer + o.r[bi].addr * w.esz);
    int rc = reduce(w.dt, w.op, src.data(), (int)src.size(), d, len, false);
    if (rc) return rc;
  }
  return 0;
}

static void post_sends(World& w, size_t me, const StageMem& ops, const uint8_t* base) {
  for (auto& o : ops) {
    if (o.peer == me) continue;
    for (auto& r : o.r)
      if (r.len > 0) w.post_send(me, o.peer, base + r.addr * w.esz, r.len);
  }
}
static void post_recvs(World& w, size_t me, const StageMem& ops, uint8_t* base) {
  for (auto& o : ops) {
    if (o.peer == me) continue;
    for (auto& r : o.r)
      if (r.len > 0) w.complete_recv(o.peer, me, base + r.addr * w.esz, r.len);
  }
}

// tree_allreduce, mpi_mod.hpp:1510-1671
static int tree(World& w, const Topo& t) {
  const size_t P = t.P, k = t.k();
  std::vector<RankPlan> plan;
  for (size_t r = 0; r < P; ++r) plan.push_back(lower(t, r, w.count));
  for (size_t i = 0; i < k; ++i) {
    for (size_t r = 0; r < P; ++r) {
      auto& rp = plan[r];
      if (!rp.send_main.empty() && !rp.send_main[i].empty())
        post_sends(w, r, rp.send_main[i], rp.send_main[i][0].from_src ? w.data[r] : w.dst[r]);
      if (!rp.send_lonely[i].empty())
        post_sends(w, r, rp.send_lonely[i], rp.send_lonely[i][0].from_src ? w.data[r] : w.dst[r]);
    }
    for (size_t r = 0; r < P; ++r) {
      auto& rp = plan[r];
      if (!rp.recv_main.empty()) post_recvs(w, r, rp.recv_main[i], w.scratch[r].data());
      if (!rp.recv_lonely[i].empty()) post_recvs(w, r, rp.recv_lonely[i], w.scratch[r].data());
    }
    for (size_t r = 0; r < P; ++r) {
      auto& rp = plan[r];
      const uint8_t* own = i == 0 ? w.data[r] : w.dst[r];
      int rc;
      if (!rp.recv_main.empty() && (rc = do_reduce(w, r, rp.recv_main[i], w.scratch[r].data(), own, w.dst[r]))) return rc;
      if (!rp.recv_lonely[i].empty() && (rc = do_reduce(w, r, rp.recv_lonely[i], w.scratch[r].data(), own, w.dst[r]))) return rc;
    }
    w.check_drained();
  }
  for (size_t i = k; i < 2 * k; ++i) {
    for (size_t r = 0; r < P; ++r) {
      auto& rp = plan[r];
      if (!rp.send_main.empty()) post_sends(w, r, rp.send_main[i], w.dst[r]);
      if (!rp.send_lonely[i].empty()) post_sends(w, r, rp.send_lonely[i], w.dst[r]);
    }
    for (size_t r = 0; r < P; ++r) {
      auto& rp = plan[r];
      if (!rp.recv_main.empty()) post_recvs(w, r, rp.recv_main[i], w.dst[r]);
      if (!rp.recv_lonely[i].empty()) post_recvs(w, r, rp.recv_lonely[i], w.dst[r]);
    }
    w.check_drained();
  }
  return 0;
}

// ring_allreduce, mpi_mod.hpp:1673-1719
static int ring(World& w) {
  const size_t P = w.P;
  std::vector<size_t> bs(P), br(P);
  for (size_t r = 0; r < P; ++r) {
    bs[r] = r;
    br[r] = (r + P - 1) % P;
  }
  auto rng = [&](size_t b) { return block_range(b, P, w.count, 0, true); };
  for (size_t step = 0; step + 1 < P; ++step) {
    for (size_t r = 0; r < P; ++r) {
      Range s = rng(bs[r]);
      if (s.len) w.post_send(r, (r + 1) % P, (step == 0 ? w.data[r] : w.dst[r]) + s.addr * w.esz, s.len);
    }
    for (size_t r = 0; r < P; ++r) {
      Range q = rng(br[r]);
      if (q.len) w.complete_recv((r + P - 1) % P, r, w.scratch[r].data() + q.addr * w.esz, q.len);
    }
    for (size_t r = 0; r < P; ++r) {
      Range q = rng(br[r]);
      if (!q.len) continue;
      const void* src[2] = {w.data[r] + q.actual * w.esz, w.scratch[r].data() + q.addr * w.esz};
      int rc = reduce(w.dt, w.op, src, 2, w.dst[r] + q.actual * w.esz, q.len, false);
      if (rc) return rc;
      }
    for (size_t r = 0; r < P; ++r) {
      bs[r] = (bs[r] + P - 1) % P;
      br[r] = (br[r] + P - 1) % P;
    }
    w.check_drained();
  }
  for (size_t step = 0; step + 1 < P; ++step) {
    for (size_t r = 0; r < P; ++r) {
      Range s = rng(bs[r]);
      if (s.len) w.post_send(r, (r + 1) % P, w.dst[r] + s.addr * w.esz, s.len);
    }
    for (size_t r = 0; r < P; ++r) {
      Range q = rng(br[r]);
      if (q.len) w.complete_recv((r + P - 1) % P, r, w.dst[r] + q.addr * w.esz, q.len);
    }
    for (size_t r = 0; r < P; ++r) {
      bs[r] = (bs[r] + P - 1) % P;
      br[r] = (br[r] + P - 1) % P;
    }
    w.check_drained();
  }
  return 0;
}

static std::string plan_json(const Topo& t, size_t n, size_t count) {
  RankPlan rp = lower(t, n, count);
  std::ostringstream os;
  auto dump = [&](const std::vector<StageMem>& v) {
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
  };
  os << "{\"send\":";
  dump(rp.send_main);
  os << ",\"send_lonely\":";
  dump(rp.send_lonely);
  os << ",\"recv\":";
  dump(rp.recv_main);
  os << ",\"recv_lonely\":";
  dump(rp.recv_lonely);
  os << "}";
  return os.str();
}

static bool make_topo(int P, const int* stages, int nstages, int lonely, Topo& t, bool& is_ring) {
  t.P = (size_t)P;
  t.L = (size_t)lonely;
  t.S = t.P - t.L;
  t.w.clear();
  is_ring = false;
  size_t pi = 1;
  for (int i = 0; i < nstages; ++i) {
    if (stages[i] == 1) {  // get_stages: any 1 => ring (mpi_mod.hpp:1461-1464)
      is_ring = true;
      t.w = {1};
      t.L = 0;
      t.S = t.P;
      return true;
    }
    t.w.push_back((size_t)stages[i]);
    pi *= (size_t)stages[i];
  }
  // validity check of get_stages (mpi_mod.hpp:1471-1475)
  if (pi + t.L != t.P || (t.L != 0 && t.w.size() < 2)) return false;
  return true;
}

}  // namespace oracle

// ============================================================================
// C ABI used by tests/ and bench.py (cpu_baseline) through ctypes.
// ============================================================================
extern "C" {

int oracle_dtype_size(int dt) { return (int)oracle::dtype_size(dt); }

// k-way reduce; copy_k1 selects vector_add/reduce_sum.h (1) or mpi_mod.hpp (0) semantics
int oracle_reduce(int dtype, int op, const void* const* srcs, int k, void* dst, size_t n, int copy_k1) {
  try {
    return oracle::reduce(dtype, op, srcs, k, dst, n, copy_k1 != 0);
  } catch (const std::exception& e) {
    fprintf(stderr, "oracle_reduce: %s\n", e.what());
    return -1;
  }
}

// Simulated MPI_Allreduce_FT over P ranks.  send[r] == NULL means MPI_IN_PLACE
// (recv[r] holds rank r's input).  Returns 0, or <0 on an invalid topology
// (the reference exit(1)s there) or an inconsistent schedule.
int oracle_allreduce(int P, const int* stages, int nstages, int lonely, int dtype, int op,
                     size_t count, const void* const* send, void* const* recv) {
  try {
    oracle::World w;
    w.P = (size_t)P;
    w.count = count;
    w.esz = oracle::dtype_size(dtype);
    w.dt = dtype;
    w.op = op;
    if (P <= 1) {  // mpi_mod.hpp:1739-1746
      if (P == 1 && send && send[0]) std::memcpy(recv[0], send[0], count * w.esz);
      return 0;
    }
    oracle::Topo t;
    bool is_ring;
    if (!oracle::make_topo(P, stages, nstages, lonely, t, is_ring)) return -10;
    const size_t split = (count + w.P - 1) / w.P;
    for (int r = 0; r < P; ++r) {
      w.dst.push_back(static_cast<uint8_t*>(recv[r]));
      w.data.push_back(send && send[r] ? static_cast<const uint8_t*>(send[r]) : static_cast<uint8_t*>(recv[r]));
      w.scratch.emplace_back(2 * split * w.P * w.esz + 16, 0);
    }
    return is_ring ? oracle::ring(w) : oracle::tree(w, t);
  } catch (const std::exception& e) {
    fprintf(stderr, "oracle_allreduce: %s\n", e.what());
    return -1;
  }
}

// JSON of the FMA-level schedule of one rank (same shape as ref_golden --schedule).
// Returns the needed length (excluding NUL); writes at most buflen bytes.
long oracle_schedule_json(int P, const int* stages, int nstages, int lonely, int rank, size_t count,
                          char* buf, size_t buflen) {
  try {
    oracle::Topo t;
    bool is_ring;
    if (!oracle::make_topo(P, stages, nstages, lonely, t, is_ring) || is_ring) return -10;
    std::string s = oracle::plan_json(t, (size_t)rank, count);
    if (buf && buflen) {
      size_t m = s.size() < buflen - 1 ? s.size() : buflen - 1;
      std::memcpy(buf, s.data(), m);
      buf[m] = 0;
    }
    return (long)s.size();
  } catch (const std::exception& e) {
    fprintf(stderr, "oracle_schedule_json: %s\n", e.what());
    return -1;
  }
}

}  // extern "C"
