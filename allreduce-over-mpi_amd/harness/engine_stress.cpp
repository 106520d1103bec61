// Random AllReduce calls through the engine's paths, every result checked, as a stress driver of its HOST
// code: every data-movement form, the ring, trees and lonely layouts, pieces from 256 B to whole blocks, empty
// and ragged buckets, six dtypes with SUM and BAND, device and host buffers, in place and out of place,
// registered buffers for the peer forms, calls captured into HIP graphs and replayed (in-process groups and
// each rank of an RCCL communicator),
// the execution model steered per group so that "auto" takes every form, error paths, and groups and
// communicators created and destroyed repeatedly.
//
// Built two ways: plainly against lib/libftar.so (csrc/Makefile: lib/ftar_engine_stress, run by
// tests/test_gpu_engine_stress.py), and against a libftar.so rebuilt with the host sanitizers only
// (tools/asan/Makefile: clang++ -fsanitize=address,undefined for the host translation units, hipcc with
// -fno-gpu-sanitize for the kernels, whose device code is untouched), where any heap misuse, use after free,
// double free or undefined behaviour in plan caches, event pools, IPC maps, the local hub or the
// execution-model cache aborts the run.
//
// Results are checked too: inputs are small integers (exact in fp32 and bf16 and in every association
// order), so the expected value of every element is the plain sum (or AND) whatever the schedule.
//
// The rccl mode runs the same random calls on P PROCESSES of one RCCL communicator each (one per rank,
// loopback sockets between them, as tests/rccl_loopback_child.py), so the RCCL transport, the first-contact
// helper thread, IPC maps of the other processes' exchange and registered buffers and communicator
// re-creation run under the sanitizers too.
//
//   engine_stress [calls] [seed]               in-process groups, default 1500 calls, seed 1
//   engine_stress rccl P calls seed [gens]     P processes, `gens` communicators one after the other
//   engine_stress host P calls seed [gens]     the same on ftar_comm_init_host (shared-memory bootstrap,
//                                              peer forms only)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include <pthread.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#include "ftar.h"

// the library's A/B knobs (exported, not in ftar.h)
extern "C" {
ftar_status_t ftar_debug_set_peer_tuning(ftar_comm_t comm, int nt, int lds);
ftar_status_t ftar_debug_set_peer_dma(ftar_comm_t comm, int dma);
ftar_status_t ftar_debug_set_rccl_register(ftar_comm_t comm, int on);
}

namespace {

#define HIP_OK(x)                                                                       \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                          \
    }                                                                                   \
  } while (0)

struct Dt {
  ftar_dtype_t t;
  size_t size;
  const char* name;
};
const Dt kDtypes[] = {{FTAR_FLOAT32, 4, "f32"}, {FTAR_BFLOAT16, 2, "bf16"}, {FTAR_INT32, 4, "i32"},
                      {FTAR_UINT8, 1, "u8"}, {FTAR_FLOAT64, 8, "f64"}, {FTAR_INT16, 2, "i16"}};

// element i of rank r: a small integer (|v| <= 8, so P = 8 sums stay exact in bf16's 8-bit mantissa)
int value(size_t i, int r) { return (int)((i * 7 + (size_t)r * 13 + (i >> 9)) % 17) - 8; }

uint16_t to_bf16(float f) {  // exact for small integers
  uint32_t u;
  memcpy(&u, &f, 4);
  return (uint16_t)(u >> 16);
}
float from_bf16(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

void fill(std::vector<uint8_t>& b, const Dt& d, size_t n, int r, bool band) {
  b.resize(n * d.size);
  for (size_t i = 0; i < n; ++i) {
    const int v = band ? (int)((i * 2654435761u + (size_t)r * 40503u) & 0x7fffffff) : value(i, r);
    switch (d.t) {
      case FTAR_FLOAT32: { float f = (float)v; memcpy(&b[i * 4], &f, 4); break; }
      case FTAR_BFLOAT16: { uint16_t h = to_bf16((float)v); memcpy(&b[i * 2], &h, 2); break; }
      case FTAR_INT32: { int32_t x = v; memcpy(&b[i * 4], &x, 4); break; }
      case FTAR_UINT8: b[i] = (uint8_t)v; break;
      case FTAR_FLOAT64: { double f = (double)v; memcpy(&b[i * 8], &f, 8); break; }
      case FTAR_INT16: { int16_t x = (int16_t)v; memcpy(&b[i * 2], &x, 2); break; }
      default: abort();
    }
  }
}

// the expected result (every rank): sum or AND of the P inputs, in the element type
// (off: the inputs of ranks off .. off + P - 1, for the graph replays' fresh inputs)
void expect(std::vector<uint8_t>& out, const Dt& d, size_t n, int P, bool band, int off = 0) {
  std::vector<std::vector<uint8_t>> ins(P);
  for (int r = 0; r < P; ++r) fill(ins[r], d, n, r + off, band);
  out.assign(n * d.size, 0);
  for (size_t i = 0; i < n; ++i) {
    switch (d.t) {
      case FTAR_FLOAT32: {
        float s = 0;
        for (int r = 0; r < P; ++r) { float f; memcpy(&f, &ins[r][i * 4], 4); s += f; }
        memcpy(&out[i * 4], &s, 4);
        break;
      }
      case FTAR_BFLOAT16: {
        float s = 0;
        for (int r = 0; r < P; ++r) { uint16_t h; memcpy(&h, &ins[r][i * 2], 2); s += from_bf16(h); }
        uint16_t h = to_bf16(s);
        memcpy(&out[i * 2], &h, 2);
        break;
      }
      case FTAR_INT32: {
        int32_t s = band ? -1 : 0;
        for (int r = 0; r < P; ++r) {
          int32_t x;
          memcpy(&x, &ins[r][i * 4], 4);
          s = band ? (s & x) : (int32_t)((uint32_t)s + (uint32_t)x);
        }
        memcpy(&out[i * 4], &s, 4);
        break;
      }
      case FTAR_UINT8: {
        uint8_t s = band ? 0xff : 0;
        for (int r = 0; r < P; ++r) s = band ? (uint8_t)(s & ins[r][i]) : (uint8_t)(s + ins[r][i]);
        out[i] = s;
        break;
      }
      case FTAR_FLOAT64: {
        double s = 0;
        for (int r = 0; r < P; ++r) { double f; memcpy(&f, &ins[r][i * 8], 8); s += f; }
        memcpy(&out[i * 8], &s, 8);
        break;
      }
      case FTAR_INT16: {
        int16_t s = band ? -1 : 0;
        for (int r = 0; r < P; ++r) {
          int16_t x;
          memcpy(&x, &ins[r][i * 2], 2);
          s = band ? (int16_t)(s & x) : (int16_t)((uint16_t)s + (uint16_t)x);
        }
        memcpy(&out[i * 2], &s, 2);
        break;
      }
      default: abort();
    }
  }
}

// every valid layout of P: the ring, each ordered factorization, and lonely L with S = P - L ranks in >= 2
// stages and L * w0 <= S (as tests/random_cases.py)
struct Layout {
  const char* topo;
  const char* lonely;
};
void factorizations(int n, std::vector<int>& cur, std::vector<std::vector<int>>& out) {
  if (n == 1) {
    if (!cur.empty()) out.push_back(cur);
    return;
  }
  for (int f = 2; f <= n; ++f)
    if (n % f == 0) {
      cur.push_back(f);
      factorizations(n / f, cur, out);
      cur.pop_back();
    }
}
std::vector<Layout> layouts(int P) {
  static std::deque<std::string> keep;  // the strings the layouts point at (stable, never freed)
  auto str = [](const std::vector<int>& f) {
    std::string t;
    for (int w : f) t += (t.empty() ? "" : ",") + std::to_string(w);
    return t;
  };
  std::vector<std::pair<std::string, int>> opts = {{"1", 0}};
  std::vector<int> cur;
  std::vector<std::vector<int>> fs;
  factorizations(P, cur, fs);
  for (auto& f : fs)
    if (f.size() <= 4) opts.push_back({str(f), 0});
  for (int L = 1; L < P; ++L) {
    std::vector<std::vector<int>> gs;
    factorizations(P - L, cur, gs);
    for (auto& f : gs)
      if (f.size() >= 2 && f.size() <= 4 && L * f[0] <= P - L) opts.push_back({str(f), L});
  }
  std::vector<Layout> out;
  for (auto& o : opts) {
    keep.push_back(o.first);
    const char* t = keep.back().c_str();
    const char* l = nullptr;
    if (o.second) {
      keep.push_back(std::to_string(o.second));
      l = keep.back().c_str();
    }
    out.push_back({t, l});
  }
  return out;
}

// one random call; every rank of a multi-process run draws the same sequence, so the settings agree
struct Case {
  Layout L;
  int form;
  size_t chunk;
  const Dt* d;
  bool band;
  size_t n;
  bool host, oop, registered;
  // per-call knobs: the peer forms' copy tuning (nt, lds, dma bits), the reduce stream's CU share, RCCL's own
  // buffer registration, phase timing, and (in-process) a user stream per rank from a small pool (-1: none)
  int tune, cus;
  bool rccl_reg, timing;
  int stream_sel;
};
Case draw(std::mt19937_64& rng, int P, const std::vector<Layout>& lay, size_t reg_bytes) {
  static const int forms[] = {FTAR_FORM_AUTO, FTAR_FORM_DIRECT, FTAR_FORM_STAGES, FTAR_FORM_COLLECTIVE,
                              FTAR_FORM_PEER_READ, FTAR_FORM_PEER_WRITE};
  static const size_t chunks[] = {0, 256, 4096 + 256, 1u << 16, 1u << 20};
  Case k;
  k.L = lay[rng() % lay.size()];
  k.form = forms[rng() % 6];
  k.chunk = chunks[rng() % 5];
  k.d = &kDtypes[rng() % 6];
  const bool integer = k.d->t == FTAR_INT32 || k.d->t == FTAR_UINT8 || k.d->t == FTAR_INT16;
  k.band = integer && rng() % 3 == 0;
  const size_t ragged = 1000 + rng() % 5000, big = 100000 + rng() % 300000;
  const size_t sizes[] = {0, 1, (size_t)P - 1, (size_t)P + 1, ragged, big};
  k.n = sizes[rng() % 6];
  k.host = rng() % 4 == 0;
  k.oop = rng() % 2 == 0;
  k.registered = !k.host && k.oop && rng() % 3 == 0;
  if (k.registered) k.n = std::min(k.n, reg_bytes / k.d->size);
  static const int cus[] = {0, 0, 32, 128};
  k.tune = (int)(rng() % 8);
  k.cus = cus[rng() % 4];
  k.rccl_reg = rng() % 4 == 0;
  k.timing = rng() % 6 == 0;
  k.stream_sel = rng() % 3 == 0 ? (int)(rng() % 2) : -1;
  return k;
}

// The execution model's constants for the next group / communicator: the defaults, or steered so that "auto"
// takes the peer forms, the collective all-gather or many small pieces (every rank draws the same preset)
void steer_model(std::mt19937_64& rng) {
  ftar_cost_params_t k{};  // all <= 0: defaults
  switch (rng() % 5) {
    case 1: k.peer_read_gbps = 5000; k.barrier_us = 1; break;
    case 2: k.peer_write_gbps = 5000; k.barrier_us = 1; break;
    case 3: k.coll_gbps = 5000; break;
    case 4: k.alpha_us = 0.05; k.issue_us = 0.05; k.link_gbps = 700; break;
    default: break;
  }
  if (ftar_cost_set(&k) != FTAR_SUCCESS) {
    fprintf(stderr, "FAIL ftar_cost_set\n");
    _Exit(1);
  }
}

// FTAR_STRESS_SKIP=dma,cus,timing,streams,tune,rcclreg: draw the knob (the call sequence stays the same) but
// leave it at its default -- to bisect a failure
bool skip(const char* knob) {
  const char* e = getenv("FTAR_STRESS_SKIP");
  return e && strstr(e, knob);
}
// On an RCCL communicator the CU share is refused (FTAR_ERR_UNSUPPORTED, the reduce stream stays on every CU:
// DESIGN §5.1); the draw still happens, so the call sequence of a seed is the same as before the rule.
void apply_knobs(ftar_comm_t c, const Case& k, bool rccl) {
  const int nt = skip("tune") ? 1 : k.tune & 1, lds = skip("tune") ? 1 : (k.tune >> 1) & 1;
  const int dma = skip("dma") ? 0 : (k.tune >> 2) & 1;
  const int cus = skip("cus") ? 0 : k.cus;
  if (rccl && cus) {
    int now = -1;
    if (ftar_comm_set_reduce_cus(c, cus) != FTAR_ERR_UNSUPPORTED || ftar_comm_get_reduce_cus(c, &now) != FTAR_SUCCESS ||
        now != 0) {
      fprintf(stderr, "FAIL reduce_cus=%d on an RCCL communicator was not refused (reduce stream on %d)\n", cus, now);
      _Exit(1);
    }
  }
  if (ftar_debug_set_peer_tuning(c, nt, lds) != FTAR_SUCCESS || ftar_debug_set_peer_dma(c, dma) != FTAR_SUCCESS ||
      ftar_comm_set_reduce_cus(c, rccl ? 0 : cus) != FTAR_SUCCESS ||
      ftar_comm_set_phase_timing(c, skip("timing") ? 0 : k.timing) != FTAR_SUCCESS ||
      (rccl && ftar_debug_set_rccl_register(c, skip("rcclreg") ? 0 : k.rccl_reg) != FTAR_SUCCESS)) {
    fprintf(stderr, "FAIL knobs: %s\n", ftar_last_error());
    _Exit(1);
  }
}

struct Stats {
  long calls = 0, checked = 0, refused = 0, groups = 0, regs = 0, captured = 0;
};

int fail(const std::string& what) {
  fprintf(stderr, "FAIL %s\n", what.c_str());
  fflush(stderr);
  _Exit(1);  // no HIP runtime static teardown under the sanitizer (see main)
}

// The call just made, captured into a HIP graph (relaxed mode; every rank's call on the capture stream, the
// form the HIP runtime ends: a stream forked per rank from the capture stream makes hipStreamEndCapture recurse
// without end, DESIGN §5.5 and profiles/r03/capture) and replayed twice on fresh inputs in the same buffers; the
// uncaptured call before it grew every buffer the plan needs
void capture_replay(int P, std::vector<ftar_comm_t>& comms, std::vector<void*>& send, std::vector<void*>& recv,
                    size_t n, const Dt& d, ftar_op_t op, bool band, const ftar_topo_t* topo, bool oop,
                    const std::string& what, Stats* st) {
  const size_t bytes = n * d.size;
  if (getenv("FTAR_STRESS_VERBOSE")) {
    fprintf(stderr, "capture: %s\n", what.c_str());
    fflush(stderr);
  }
  hipStream_t s0;
  HIP_OK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  HIP_OK(hipStreamBeginCapture(s0, hipStreamCaptureModeRelaxed));
  std::vector<void*> rsv(P, (void*)s0);
  const ftar_status_t s = ftar_allreduce_group(oop ? send.data() : nullptr, recv.data(), n, d.t, op, topo,
                                               comms.data(), P, rsv.data());
  const std::string err = s == FTAR_SUCCESS ? "" : ftar_last_error();
  hipGraph_t g = nullptr;
  const hipError_t e = hipStreamEndCapture(s0, &g);
  if (s != FTAR_SUCCESS) fail(what + ": captured call: " + ftar_status_string(s) + ": " + err);
  if (e != hipSuccess) fail(what + ": hipStreamEndCapture: " + hipGetErrorString(e));
  hipGraphExec_t x;
  HIP_OK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
  for (int rep = 1; rep <= 2; ++rep) {
    std::vector<uint8_t> in, want, got(bytes);
    for (int r = 0; r < P; ++r) {
      fill(in, d, n, r + 7 * rep, band);
      HIP_OK(hipMemcpy(oop ? send[r] : recv[r], in.data(), bytes, hipMemcpyHostToDevice));
      if (oop) HIP_OK(hipMemset(recv[r], 0x5a, bytes));
    }
    HIP_OK(hipDeviceSynchronize());  // s0 is non-blocking: the legacy-stream writes above must be done first
    HIP_OK(hipGraphLaunch(x, s0));
    HIP_OK(hipStreamSynchronize(s0));
    expect(want, d, n, P, band, 7 * rep);
    for (int r = 0; r < P; ++r) {
      HIP_OK(hipMemcpy(got.data(), recv[r], bytes, hipMemcpyDeviceToHost));
      if (got != want) fail(what + ": graph replay " + std::to_string(rep) + ": rank " + std::to_string(r) + " differs");
    }
  }
  ++st->captured;
  HIP_OK(hipGraphExecDestroy(x));
  HIP_OK(hipGraphDestroy(g));
  HIP_OK(hipStreamDestroy(s0));
}

// one group: `calls` random calls, then destroyed
void run_group(int P, int calls, std::mt19937_64& rng, Stats* st) {
  steer_model(rng);
  std::vector<ftar_comm_t> comms(P);
  std::vector<int> devs(P, 0);
  if (ftar_comm_init_local(comms.data(), P, devs.data()) != FTAR_SUCCESS) fail(std::string("init_local: ") + ftar_last_error());
  ++st->groups;
  std::vector<void*> pool(2 * P);
  for (auto& q : pool) HIP_OK(hipStreamCreateWithFlags(reinterpret_cast<hipStream_t*>(&q), hipStreamNonBlocking));
  const auto lay = layouts(P);
  // registered device buffers (the peer forms' no-copy path): one pair per rank, registered collectively
  const size_t reg_bytes = 1u << 22;
  std::vector<void*> rx(P), ry(P);
  std::vector<int> idx(P), idy(P);
  for (int r = 0; r < P; ++r) {
    HIP_OK(hipMalloc(&rx[r], reg_bytes));
    HIP_OK(hipMalloc(&ry[r], reg_bytes));
  }
  {
    std::vector<std::thread> th;
    std::vector<ftar_status_t> s(P);
    for (int r = 0; r < P; ++r)
      th.emplace_back([&, r] {
        s[r] = ftar_comm_register(comms[r], rx[r], reg_bytes, &idx[r]);
        if (s[r] == FTAR_SUCCESS) s[r] = ftar_comm_register(comms[r], ry[r], reg_bytes, &idy[r]);
      });
    for (auto& t : th) t.join();
    for (int r = 0; r < P; ++r)
      if (s[r] != FTAR_SUCCESS) fail(std::string("register: ") + ftar_last_error());
    st->regs += 2 * P;
  }
  for (int call = 0; call < calls; ++call) {
    const Case k = draw(rng, P, lay, reg_bytes);
    const Layout L = k.L;
    const int form = k.form;
    const size_t chunk = k.chunk;
    const Dt& d = *k.d;
    const bool band = k.band, host = k.host, oop = k.oop, registered = k.registered;
    const size_t n = k.n;
    ftar_topo_t topo;
    if (ftar_topo_parse(L.topo, L.lonely, P, &topo) != FTAR_SUCCESS) fail(std::string("topo_parse ") + L.topo);
    for (int r = 0; r < P; ++r) {
      if (ftar_comm_set_form(comms[r], form) != FTAR_SUCCESS) fail("set_form");
      if (ftar_comm_set_chunk_bytes(comms[r], chunk) != FTAR_SUCCESS) fail("set_chunk_bytes");
      if (ftar_comm_set_host_chunk_bytes(comms[r], chunk) != FTAR_SUCCESS) fail("set_host_chunk_bytes");
      apply_knobs(comms[r], k, false);
    }
    std::vector<void*> user_streams;  // one of two streams per rank (calls alternate streams unsynchronised)
    if (k.stream_sel >= 0 && !skip("streams"))
      for (int r = 0; r < P; ++r) user_streams.push_back(pool[2 * r + k.stream_sel]);
    const size_t bytes = n * d.size;
    std::vector<std::vector<uint8_t>> in(P);
    for (int r = 0; r < P; ++r) fill(in[r], d, n, r, band);
    std::vector<void*> send(P, nullptr), recv(P, nullptr);
    std::vector<void*> owned;
    std::vector<std::vector<uint8_t>> hbuf(2 * P);
    for (int r = 0; r < P; ++r) {
      if (host) {
        hbuf[2 * r] = in[r];
        hbuf[2 * r + 1].assign(bytes, 0x5a);
        send[r] = oop ? (void*)hbuf[2 * r].data() : nullptr;
        recv[r] = oop ? (void*)hbuf[2 * r + 1].data() : (void*)hbuf[2 * r].data();
        if (!bytes) recv[r] = send[r] = nullptr;
        continue;
      }
      void *a = nullptr, *b = nullptr;
      if (registered) {
        a = rx[r];
        b = ry[r];
      } else {
        HIP_OK(hipMalloc(&a, bytes ? bytes : 1));
        owned.push_back(a);
        if (oop) {
          HIP_OK(hipMalloc(&b, bytes ? bytes : 1));
          owned.push_back(b);
        }
      }
      if (bytes) HIP_OK(hipMemcpy(a, in[r].data(), bytes, hipMemcpyHostToDevice));
      if (oop && bytes) HIP_OK(hipMemset(b, 0x5a, bytes));
      send[r] = oop ? a : nullptr;
      recv[r] = oop ? b : a;
    }
    const ftar_op_t op = band ? FTAR_BAND : FTAR_SUM;
    void* const* sv = user_streams.empty() ? nullptr : user_streams.data();
    const ftar_status_t s = host ? ftar_allreduce_host_group(send.data(), recv.data(), n, d.t, op, &topo,
                                                             comms.data(), P, sv)
                                 : ftar_allreduce_group(send.data(), recv.data(), n, d.t, op, &topo, comms.data(),
                                                        P, sv);
    HIP_OK(hipDeviceSynchronize());
    ++st->calls;
    char what[256];
    snprintf(what, sizeof what,
             "P=%d topo=%s+%s form=%d chunk=%zu %s %s n=%zu host=%d oop=%d reg=%d tune=%d cus=%d timing=%d stream=%d",
             P, L.topo, L.lonely ? L.lonely : "0", form, chunk, d.name, band ? "band" : "sum", n, host, oop, registered,
             k.tune, k.cus, (int)k.timing, k.stream_sel);
    if (s != FTAR_SUCCESS) {
      // refusals the engine documents: forms a layout cannot take are replaced, so only errors remain
      fail(std::string(what) + ": " + ftar_status_string(s) + ": " + ftar_last_error());
    }
    std::vector<uint8_t> want;
    expect(want, d, n, P, band);
    for (int r = 0; r < P; ++r) {
      std::vector<uint8_t> got(bytes);
      if (host) got = oop ? hbuf[2 * r + 1] : hbuf[2 * r];
      else if (bytes) HIP_OK(hipMemcpy(got.data(), recv[r], bytes, hipMemcpyDeviceToHost));
      if (got != want) {
        size_t i = 0;
        while (i < bytes && got[i] == want[i]) ++i;
        fail(std::string(what) + ": rank " + std::to_string(r) + " differs at byte " + std::to_string(i));
      }
    }
    ++st->checked;
    // now and then the same call again, captured into a graph and replayed
    if (!host && bytes && rng() % 8 == 0) capture_replay(P, comms, send, recv, n, d, op, band, &topo, oop, what, st);
    for (void* p : owned) HIP_OK(hipFree(p));
  }
  // error paths: refused before anything is enqueued, the group stays usable
  {
    ftar_topo_t bad;
    if (ftar_topo_parse("3,3", nullptr, P, &bad) == FTAR_SUCCESS) {
      std::vector<void*> recv(P, rx[0]);
      for (int r = 0; r < P; ++r) recv[r] = rx[r];
      if (ftar_allreduce_group(nullptr, recv.data(), 64, FTAR_FLOAT32, FTAR_SUM, &bad, comms.data(), P, nullptr) ==
          FTAR_SUCCESS)
        fail("topology 3,3 accepted");
      ++st->refused;
    }
    std::vector<void*> recv(P);
    for (int r = 0; r < P; ++r) recv[r] = rx[r];
    if (ftar_allreduce_group(nullptr, recv.data(), 64, FTAR_FLOAT32, FTAR_BAND, nullptr, comms.data(), P, nullptr) !=
        FTAR_ERR_UNSUPPORTED)
      fail("BAND on fp32 not refused");
    ++st->refused;
  }
  for (int r = 0; r < P; ++r) {
    ftar_comm_deregister(comms[r], idx[r]);
    ftar_comm_deregister(comms[r], idy[r]);
  }
  for (int r = 0; r < P; ++r)
    if (ftar_comm_destroy(comms[r]) != FTAR_SUCCESS) fail(std::string("destroy: ") + ftar_last_error());
  for (int r = 0; r < P; ++r) {
    HIP_OK(hipFree(rx[r]));
    HIP_OK(hipFree(ry[r]));
  }
  for (auto q : pool) HIP_OK(hipStreamDestroy(static_cast<hipStream_t>(q)));
}

std::string show(const Dt& d, const uint8_t* p) {
  char b[64];
  switch (d.t) {
    case FTAR_FLOAT32: { float f; memcpy(&f, p, 4); snprintf(b, sizeof b, "%g", f); break; }
    case FTAR_BFLOAT16: { uint16_t h; memcpy(&h, p, 2); snprintf(b, sizeof b, "%g", from_bf16(h)); break; }
    case FTAR_FLOAT64: { double f; memcpy(&f, p, 8); snprintf(b, sizeof b, "%g", f); break; }
    case FTAR_INT32: { int32_t x; memcpy(&x, p, 4); snprintf(b, sizeof b, "%d", x); break; }
    case FTAR_INT16: { int16_t x; memcpy(&x, p, 2); snprintf(b, sizeof b, "%d", x); break; }
    default: snprintf(b, sizeof b, "%u", (unsigned)*p);
  }
  return b;
}

// ---- rccl mode: one process per rank ---------------------------------------------------------------------

bool read_all(int fd, void* p, size_t n) {
  auto* b = (uint8_t*)p;
  while (n) {
    const ssize_t k = read(fd, b, n);
    if (k <= 0) return false;
    b += k;
    n -= (size_t)k;
  }
  return true;
}

// the host transport's bootstrap collective (ftar_comm_init_host): an all-gather through memory shared by
// the forked ranks, two process-shared barriers per call
struct Shm {
  pthread_barrier_t bar;
  size_t cap;
  char data[1];
};
struct HostCtx {
  Shm* shm;
  int rank, P;
};
int shm_allgather(const void* mine, void* all, size_t bytes, void* user) {
  auto* h = static_cast<HostCtx*>(user);
  if (bytes * (size_t)h->P > h->shm->cap) return 1;
  memcpy(h->shm->data + (size_t)h->rank * bytes, mine, bytes);
  pthread_barrier_wait(&h->shm->bar);
  memcpy(all, h->shm->data, bytes * (size_t)h->P);
  pthread_barrier_wait(&h->shm->bar);
  return 0;
}

// rank r of P: `gens` communicators in turn, `calls` random calls on each.  rccl: ids[q] is the pipe rank 0
// writes each generation's unique id to for rank q.  host (shm != null): ftar_comm_init_host over the shared
// memory all-gather; that transport moves data by the peer forms only, on one-round plans
int rccl_rank(int r, int P, long calls, unsigned long seed, int gens, const std::vector<int>& id_pipes,
              Shm* shm = nullptr) {
  const std::string host = "ftar-stress-" + std::to_string(r);
  setenv("NCCL_HOSTID", host.c_str(), 1);
  setenv("NCCL_SOCKET_IFNAME", "lo", 1);
  setenv("NCCL_IB_DISABLE", "1", 1);
  HIP_OK(hipSetDevice(0));
  std::mt19937_64 rng(seed);  // the same sequence on every rank
  const auto lay = layouts(P);
  const size_t reg_bytes = 1u << 22;
  long checked = 0, refused = 0, captured = 0;
  for (int g = 0; g < gens; ++g) {
    steer_model(rng);  // before the communicator's first call, where the ranks compare the constants
    ftar_comm_t c;
    HostCtx hctx{shm, r, P};
    if (shm) {
      if (ftar_comm_init_host(&c, P, r, 0, shm_allgather, &hctx) != FTAR_SUCCESS)
        fail(std::string("init_host: ") + ftar_last_error());
    } else {
      ftar_unique_id_t id;
      if (r == 0) {
        if (ftar_get_unique_id(&id) != FTAR_SUCCESS) fail(std::string("get_unique_id: ") + ftar_last_error());
        for (int q = 1; q < P; ++q)
          if (write(id_pipes[q], &id, sizeof id) != (ssize_t)sizeof id) fail("id pipe write");
      } else if (!read_all(id_pipes[r], &id, sizeof id)) {
        fail("id pipe read");
      }
      if (ftar_comm_init_rank(&c, P, id, r, 0) != FTAR_SUCCESS) fail(std::string("init_rank: ") + ftar_last_error());
    }
    void *rx, *ry;
    int idx, idy;
    HIP_OK(hipMalloc(&rx, reg_bytes));
    HIP_OK(hipMalloc(&ry, reg_bytes));
    if (ftar_comm_register(c, rx, reg_bytes, &idx) != FTAR_SUCCESS ||
        ftar_comm_register(c, ry, reg_bytes, &idy) != FTAR_SUCCESS)
      fail(std::string("register: ") + ftar_last_error());
    for (long call = 0; call < calls; ++call) {
      Case k = draw(rng, P, lay, reg_bytes);
      if (shm) {  // the host transport: peer forms on one-round plans (no lonely ranks)
        k.form = (k.form & 1) ? FTAR_FORM_PEER_READ : FTAR_FORM_PEER_WRITE;
        if (k.L.lonely) k.L = {"1", nullptr};
      }
      const Dt& d = *k.d;
      const size_t bytes = k.n * d.size;
      ftar_topo_t topo;
      if (ftar_topo_parse(k.L.topo, k.L.lonely, P, &topo) != FTAR_SUCCESS) fail("topo_parse");
      if (ftar_comm_set_form(c, k.form) != FTAR_SUCCESS || ftar_comm_set_chunk_bytes(c, k.chunk) != FTAR_SUCCESS ||
          ftar_comm_set_host_chunk_bytes(c, k.chunk) != FTAR_SUCCESS)
        fail("setters");
      apply_knobs(c, k, !shm);
      std::vector<uint8_t> in, hout;
      fill(in, d, k.n, r, k.band);
      void *send = nullptr, *recv = nullptr, *a = nullptr, *b = nullptr;
      if (k.host) {
        hout.assign(bytes, 0x5a);
        send = k.oop ? (void*)in.data() : nullptr;
        recv = k.oop ? (void*)hout.data() : (void*)in.data();
        if (!bytes) send = recv = nullptr;
      } else {
        if (k.registered) {
          a = rx;
          b = ry;
        } else {
          HIP_OK(hipMalloc(&a, bytes ? bytes : 1));
          if (k.oop) HIP_OK(hipMalloc(&b, bytes ? bytes : 1));
        }
        if (bytes) HIP_OK(hipMemcpy(a, in.data(), bytes, hipMemcpyHostToDevice));
        if (k.oop && bytes) HIP_OK(hipMemset(b, 0x5a, bytes));
        send = k.oop ? a : nullptr;
        recv = k.oop ? b : a;
      }
      const ftar_op_t op = k.band ? FTAR_BAND : FTAR_SUM;
      if (getenv("FTAR_STRESS_VERBOSE")) {
        fprintf(stderr, "rank %d gen %d call %ld: topo=%s+%s form=%d chunk=%zu %s n=%zu host=%d oop=%d reg=%d tune=%d "
                "cus=%d timing=%d rcclreg=%d\n", r, g, call, k.L.topo, k.L.lonely ? k.L.lonely : "0", k.form, k.chunk,
                d.name, k.n, k.host, k.oop, k.registered, k.tune, k.cus, (int)k.timing, (int)k.rccl_reg);
        fflush(stderr);
      }
      const ftar_status_t s = k.host ? ftar_allreduce_host(send, recv, k.n, d.t, op, &topo, c, nullptr)
                                     : ftar_allreduce(send, recv, k.n, d.t, op, &topo, c, nullptr);
      HIP_OK(hipDeviceSynchronize());
      char what[256];
      snprintf(what, sizeof what, "rank %d gen %d call %ld: topo=%s+%s form=%d chunk=%zu %s %s n=%zu host=%d oop=%d "
               "reg=%d", r, g, call, k.L.topo, k.L.lonely ? k.L.lonely : "0", k.form, k.chunk, d.name,
               k.band ? "band" : "sum", k.n, k.host, k.oop, k.registered);
      if (s != FTAR_SUCCESS) fail(std::string(what) + ": " + ftar_status_string(s) + ": " + ftar_last_error());
      std::vector<uint8_t> got(bytes), want;
      if (k.host) got = k.oop ? hout : in;
      else if (bytes) HIP_OK(hipMemcpy(got.data(), recv, bytes, hipMemcpyDeviceToHost));
      expect(want, d, k.n, P, k.band);
      if (got != want) {
        std::string diff;
        int shown = 0;
        for (size_t i = 0; i < k.n && shown < 12; ++i)
          if (memcmp(&got[i * d.size], &want[i * d.size], d.size)) {
            diff += " [" + std::to_string(i) + "] got " + show(d, &got[i * d.size]) + " want " +
                    show(d, &want[i * d.size]);
            ++shown;
          }
        fail(std::string(what) + ": differs from the exact result:" + diff);
      }
      ++checked;
      // now and then the same call captured into a HIP graph on this rank (every rank alike: the product's
      // process model under capture) and replayed twice on fresh inputs; the graphs meet through RCCL
      if (!k.host && bytes && !shm && rng() % 8 == 0) {
        hipStream_t cs;
        HIP_OK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
        HIP_OK(hipStreamBeginCapture(cs, hipStreamCaptureModeRelaxed));
        const ftar_status_t s2 = ftar_allreduce(send, recv, k.n, d.t, op, &topo, c, cs);
        const std::string err2 = s2 == FTAR_SUCCESS ? "" : ftar_last_error();
        hipGraph_t gr = nullptr;
        const hipError_t e2 = hipStreamEndCapture(cs, &gr);
        if (s2 != FTAR_SUCCESS) fail(std::string(what) + ": captured call: " + ftar_status_string(s2) + ": " + err2);
        if (e2 != hipSuccess) fail(std::string(what) + ": hipStreamEndCapture: " + hipGetErrorString(e2));
        hipGraphExec_t gx;
        HIP_OK(hipGraphInstantiate(&gx, gr, nullptr, nullptr, 0));
        for (int rep = 1; rep <= 2; ++rep) {
          std::vector<uint8_t> in2, want2, got2(bytes);
          fill(in2, d, k.n, r + 7 * rep, k.band);
          HIP_OK(hipMemcpy(k.oop ? send : recv, in2.data(), bytes, hipMemcpyHostToDevice));
          if (k.oop) HIP_OK(hipMemset(recv, 0x5a, bytes));
          HIP_OK(hipDeviceSynchronize());
          HIP_OK(hipGraphLaunch(gx, cs));
          HIP_OK(hipStreamSynchronize(cs));
          HIP_OK(hipMemcpy(got2.data(), recv, bytes, hipMemcpyDeviceToHost));
          expect(want2, d, k.n, P, k.band, 7 * rep);
          if (got2 != want2) fail(std::string(what) + ": graph replay " + std::to_string(rep) + " differs");
        }
        HIP_OK(hipGraphExecDestroy(gx));
        HIP_OK(hipGraphDestroy(gr));
        HIP_OK(hipStreamDestroy(cs));
        ++captured;
      }
      if (r == 0 && checked % 25 == 0) {  // progress (a silent run is taken to be hung)
        printf("progress: rank 0 gen %d, %ld calls checked\n", g, checked);
        fflush(stdout);
      }
      if (!k.host && !k.registered) {
        HIP_OK(hipFree(a));
        if (b) HIP_OK(hipFree(b));
      }
    }
    // refused alike on every rank before anything is enqueued; the communicator stays usable
    if (ftar_allreduce(nullptr, rx, 64, FTAR_FLOAT32, FTAR_BAND, nullptr, c, nullptr) != FTAR_ERR_UNSUPPORTED)
      fail("BAND on fp32 not refused");
    ++refused;
    ftar_comm_deregister(c, idx);
    ftar_comm_deregister(c, idy);
    if (ftar_comm_destroy(c) != FTAR_SUCCESS) fail(std::string("destroy: ") + ftar_last_error());
    HIP_OK(hipFree(rx));
    HIP_OK(hipFree(ry));
  }
  printf("{\"rank\": %d, \"checked\": %ld, \"captured\": %ld, \"refused\": %ld, \"communicators\": %d}\n", r, checked,
         captured, refused, gens);
  fflush(stdout);
  HIP_OK(hipDeviceSynchronize());
  _Exit(0);  // as in main: no HIP runtime static teardown under the sanitizer
}

// forks the P ranks BEFORE anything in this process touches HIP; returns 0 when every rank exits 0
int rccl_main(int P, long calls, unsigned long seed, int gens, bool host = false) {
  Shm* shm = nullptr;
  if (host) {
    const size_t cap = 4u << 20;
    void* m = mmap(nullptr, sizeof(Shm) + cap, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    if (m == MAP_FAILED) fail("mmap");
    shm = static_cast<Shm*>(m);
    shm->cap = cap;
    pthread_barrierattr_t a;
    pthread_barrierattr_init(&a);
    pthread_barrierattr_setpshared(&a, PTHREAD_PROCESS_SHARED);
    pthread_barrier_init(&shm->bar, &a, (unsigned)P);
  }
  std::vector<int> rd(P, -1), wr(P, -1);
  for (int q = 1; q < P; ++q) {
    int fd[2];
    if (pipe(fd)) fail("pipe");
    rd[q] = fd[0];
    wr[q] = fd[1];
  }
  std::vector<pid_t> pids;
  for (int r = 0; r < P; ++r) {
    const pid_t pid = fork();
    if (pid < 0) fail("fork");
    if (pid == 0) {
      std::vector<int> mine(P, -1);
      for (int q = 1; q < P; ++q) mine[q] = r == 0 ? wr[q] : (q == r ? rd[q] : -1);
      return rccl_rank(r, P, calls, seed, gens, mine, shm);
    }
    pids.push_back(pid);
  }
  // the first rank to fail ends the run: its peers would wait for it in their next call forever
  int worst = 0;
  size_t left = pids.size();
  while (left) {
    int status = 0;
    const pid_t pid = waitpid(-1, &status, 0);
    if (pid < 0) break;
    --left;
    const int code = WIFEXITED(status) ? WEXITSTATUS(status) : 128 + WTERMSIG(status);
    worst = std::max(worst, code);
    if (code) {
      usleep(500000);  // let the other ranks report the same call
      for (pid_t q : pids)
        if (q != pid) kill(q, SIGKILL);
    }
  }
  printf("%s: P=%d calls=%ld seed=%lu communicators=%d: %s\n", host ? "host" : "rccl", P, calls, seed, gens,
         worst ? "FAILED" : "ok");
  return worst;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc > 1 && (!strcmp(argv[1], "rccl") || !strcmp(argv[1], "host"))) {
    if (argc < 5) {
      fprintf(stderr, "usage: engine_stress rccl|host P calls seed [gens]\n");
      return 2;
    }
    return rccl_main(atoi(argv[2]), atol(argv[3]), strtoul(argv[4], nullptr, 0), argc > 5 ? atoi(argv[5]) : 2,
                     !strcmp(argv[1], "host"));
  }
  const long total = argc > 1 ? atol(argv[1]) : 1500;
  const unsigned long seed = argc > 2 ? strtoul(argv[2], nullptr, 0) : 1;
  HIP_OK(hipSetDevice(0));
  std::mt19937_64 rng(seed);
  Stats st;
  const int worlds[] = {2, 3, 4, 5, 6, 8};
  long done = 0;
  int round = 0;
  while (done < total) {
    const int P = worlds[round++ % 6];
    const int calls = 20 + (int)(rng() % 60);  // groups come and go: bring-up and teardown under ASan too
    run_group(P, calls, rng, &st);
    done += calls;
    if (round % 6 == 0) {
      printf("progress: %ld calls, %ld groups\n", st.calls, st.groups);
      fflush(stdout);
    }
  }
  printf("{\"calls\": %ld, \"checked\": %ld, \"captured\": %ld, \"refused\": %ld, \"groups\": %ld, "
         "\"registrations\": %ld, \"seed\": %lu}\n",
         st.calls, st.checked, st.captured, st.refused, st.groups, st.regs, seed);
  fflush(stdout);
  // every group is destroyed and the device drained; skip the HIP runtime's static teardown, where the
  // sanitizer's own HIP allocator hooks trip a CHECK once the runtime has unloaded (not ftar code)
  HIP_OK(hipDeviceSynchronize());
  _Exit(0);
}
