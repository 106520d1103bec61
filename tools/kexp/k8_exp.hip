// k-way reduce kernel experiments (fp32 sum), cold data: launches rotate over
// S disjoint (k sources + destination) sets so nothing is served by the MALL.
// Standalone: hipcc --offload-arch=gfx950 -O3 -std=c++17 k8_exp.hip -o k8_exp
//   ./k8_exp [k] [elements] [sets] [reps] [rounds]
// Every variant's output is compared bit for bit with variant 0 (the
// production LDS-staged kernel's structure).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int K>
struct Srcs {
  const f32x4* p[K];
};

#define GPTR(p) ((__attribute__((address_space(1))) void*)(p))
#define LPTR(p) ((__attribute__((address_space(3))) void*)(p))

__device__ __forceinline__ void st_nt(f32x4* p, f32x4 v) { __builtin_nontemporal_store(v, p); }

// gfx9 s_waitcnt encoding: vmcnt N (0..63), expcnt and lgkmcnt not waited on
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// ---- variant 0: production structure: every wave DMAs U tiles of all K sources, waits for all, folds
template <int K, int U, int W = 4>
__global__ void __launch_bounds__(W * 64) k_lds(Srcs<K> src, f32x4* dst, size_t nvec) {
  __shared__ f32x4 lds[W][K][U][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t base = ((size_t)blockIdx.x * W + wave) * (U * 64);
  if (base + U * 64 > nvec) return;
#pragma unroll
  for (int j = 0; j < K; ++j)
#pragma unroll
    for (int u = 0; u < U; ++u)
      __builtin_amdgcn_global_load_lds(GPTR(src.p[j] + base + u * 64 + lane), LPTR(&lds[wave][j][u][0]), 16, 0, 2);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int u = 0; u < U; ++u) {
    f32x4 a = lds[wave][0][u][lane];
#pragma unroll
    for (int j = 1; j < K; ++j) a += lds[wave][j][u][lane];
    st_nt(dst + base + u * 64 + lane, a);
  }
}

// ---- variant 1: source ring.  Each wave owns U consecutive tiles (U KiB contiguous per
// source); D sources in flight in an LDS ring of D slots; accumulators in VGPRs.  Loads of
// source j+D are issued as soon as source j has been folded.  LDS per WG = W*D*U KiB,
// independent of K.
template <int K, int U, int D, int W>
__global__ void __launch_bounds__(W * 64) k_ring(Srcs<K> src, f32x4* dst, size_t nvec) {
  __shared__ f32x4 lds[W][D][U][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t base = ((size_t)blockIdx.x * W + wave) * (U * 64);
  if (base + U * 64 > nvec) return;
#pragma unroll
  for (int j = 0; j < D && j < K; ++j)
#pragma unroll
    for (int u = 0; u < U; ++u)
      __builtin_amdgcn_global_load_lds(GPTR(src.p[j] + base + u * 64 + lane), LPTR(&lds[wave][j][u][0]), 16, 0, 2);
  f32x4 acc[U];
  auto step = [&](auto jc) {
    constexpr int j = decltype(jc)::value;
    constexpr int ahead = (K - 1 - j) < (D - 1) ? (K - 1 - j) : (D - 1);  // sources issued after j
    wait_vm<ahead * U>();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const f32x4 x = lds[wave][j % D][u][lane];
      acc[u] = j == 0 ? x : acc[u] + x;
    }
    if constexpr (j + D < K) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot j%D read before it is refilled
#pragma unroll
      for (int u = 0; u < U; ++u)
        __builtin_amdgcn_global_load_lds(GPTR(src.p[j + D] + base + u * 64 + lane), LPTR(&lds[wave][j % D][u][0]), 16,
                                         0, 2);
    }
  };
  [&]<int... J>(std::integer_sequence<int, J...>) { (step(std::integral_constant<int, J>{}), ...); }
  (std::make_integer_sequence<int, K>{});
#pragma unroll
  for (int u = 0; u < U; ++u) st_nt(dst + base + u * 64 + lane, acc[u]);
}

// ---- variant 2: register-only, all K x U loads in flight, W waves
template <int K, int U, int W>
__global__ void __launch_bounds__(W * 64) k_reg(Srcs<K> src, f32x4* dst, size_t nvec) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t base = ((size_t)blockIdx.x * W + wave) * (U * 64);
  if (base + U * 64 > nvec) return;
  f32x4 x[K][U];
#pragma unroll
  for (int j = 0; j < K; ++j)
#pragma unroll
    for (int u = 0; u < U; ++u) x[j][u] = __builtin_nontemporal_load(src.p[j] + base + u * 64 + lane);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    f32x4 a = x[0][u];
#pragma unroll
    for (int j = 1; j < K; ++j) a += x[j][u];
    st_nt(dst + base + u * 64 + lane, a);
  }
}

// ---- variant 3: the source ring, persistent over regions: a wave walks regions grid-stride and
// keeps the ring full across region boundaries (the next region's first D sources are issued
// while the current region's last sources are folded).
template <int K, int U, int D, int W>
__global__ void __launch_bounds__(W * 64) k_ring_p(Srcs<K> src, f32x4* dst, size_t nvec) {
  static_assert(D <= K, "ring deeper than k");
  __shared__ f32x4 lds[W][D][U][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t nreg = nvec / (U * 64);
  const size_t stride = (size_t)gridDim.x * W;
  size_t r = (size_t)blockIdx.x * W + wave;
  if (r >= nreg) return;
  auto issue = [&](int j, size_t reg, int slot) {
#pragma unroll
    for (int u = 0; u < U; ++u)
      __builtin_amdgcn_global_load_lds(GPTR(src.p[j] + reg * (U * 64) + u * 64 + lane), LPTR(&lds[wave][slot][u][0]),
                                       16, 0, 2);
  };
#pragma unroll
  for (int j = 0; j < D; ++j) issue(j, r, j);
  for (; r < nreg; r += stride) {
    const size_t rn = r + stride;
    const bool more = rn < nreg;  // wave-uniform
    f32x4 acc[U];
    auto step = [&](auto jc) {
      constexpr int j = decltype(jc)::value;
      // loads issued after source j: the rest of this region's ring, then (if more) the next
      // region's first sources as they are refilled.  Counting only loads of THIS region after j
      // is conservative when the next region's loads come after them.
      constexpr int ahead = (K - 1 - j) < (D - 1) ? (K - 1 - j) : (D - 1);
      if (more) wait_vm<(D - 1) * U>();
      else wait_vm<ahead * U>();
      asm volatile("" ::: "memory");
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const f32x4 x = lds[wave][j % D][u][lane];
        acc[u] = j == 0 ? x : acc[u] + x;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if constexpr (j + D < K) issue(j + D, r, j % D);
      else if (more) issue(j + D - K, rn, j % D);
    };
    [&]<int... J>(std::integer_sequence<int, J...>) { (step(std::integral_constant<int, J>{}), ...); }
    (std::make_integer_sequence<int, K>{});
#pragma unroll
    for (int u = 0; u < U; ++u) st_nt(dst + r * (U * 64) + u * 64 + lane, acc[u]);
  }
}

// ---- variant 4: progressive: loads issued tile-major, tile u folded and stored as soon as its K
// loads have landed (counted vmcnt; loads return in order, so stores in the count only make a
// wait longer), while tiles u+1.. are still in flight
// store policies: 0 nt (production), 1 plain, 2 sc1, 3 sc0 sc1, 4 sc1 nt
template <int ST>
__device__ __forceinline__ void st_pol(f32x4* p, f32x4 v) {
  if constexpr (ST == 0) __builtin_nontemporal_store(v, p);
  else if constexpr (ST == 1) *p = v;
  else if constexpr (ST == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  else if constexpr (ST == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
  else asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
}

// issue order of the K sources (the fold still reads them 0..K-1 from LDS):
//   ORD 0 ascending (production); 1 wave parity: odd waves descending; 2 block parity: odd blocks
//   descending; 3 rotated by blockIdx % K (every source is somebody's first at any moment)
// BURST: fold every tile as it lands but keep the results in registers and store all U tiles at the end
template <int K, int R>
__device__ __forceinline__ constexpr int rot(int j) { return (j + R) % K; }

template <int K, int U, int W, int SW = 0, bool RO = false, int ST = 0, int ORD = 0, bool BURST = false>
__global__ void __launch_bounds__(W * 64) k_prog(Srcs<K> src, f32x4* dst, size_t nvec) {
  __shared__ f32x4 lds[W][U][K][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  size_t b = blockIdx.x;
  if constexpr (SW == 1) {  // XCD-contiguous: blocks b and b+8 share an XCD; give each XCD one contiguous 1/8
    const size_t per = gridDim.x / 8;
    if (b < per * 8) b = (b % 8) * per + b / 8;
  } else if constexpr (SW == 2) {  // XCD-chunked: runs of 8 consecutive tiles per XCD
    const size_t g = b / 64, r = b % 64;
    if ((g + 1) * 64 <= gridDim.x) b = g * 64 + (r % 8) * 8 + r / 8;
  } else if constexpr (SW >= 3) {  // R regions interleaved: block b works in region b % R, so the
    // workgroups resident at one time stream from R distant places of every buffer (R x the streams)
    constexpr size_t R = SW == 3 ? 2 : SW == 4 ? 4 : 8;
    const size_t per = gridDim.x / R;
    if (b < per * R) b = (b % R) * per + b / R;
  }
  const size_t base = (b * W + wave) * (U * 64);
  if (base + U * 64 > nvec) return;
  auto issue = [&](auto rc, auto dc) {
    constexpr int R = decltype(rc)::value;
    constexpr bool desc = decltype(dc)::value;
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int jj = 0; jj < K; ++jj) {
        const int j = desc ? K - 1 - jj : (jj + R) % K;
        __builtin_amdgcn_global_load_lds(GPTR(src.p[j] + base + u * 64 + lane), LPTR(&lds[wave][u][j][0]), 16, 0,
                                         2);
      }
  };
  if constexpr (ORD == 0) {
    issue(std::integral_constant<int, 0>{}, std::false_type{});
  } else if constexpr (ORD == 1 || ORD == 2) {
    const bool odd = ORD == 1 ? (wave & 1) : (blockIdx.x & 1);
    if (odd) issue(std::integral_constant<int, 0>{}, std::true_type{});
    else issue(std::integral_constant<int, 0>{}, std::false_type{});
  } else {
    const int r = (int)(blockIdx.x % K);
    [&]<int... Rs>(std::integer_sequence<int, Rs...>) {
      ((r == Rs ? (issue(std::integral_constant<int, Rs>{}, std::false_type{}), 0) : 0), ...);
    }(std::make_integer_sequence<int, K>{});
  }
  if constexpr (RO) {  // read-only ceiling: the loads land in LDS, nothing is folded or stored
    wait_vm<0>();
    return;
  }
  f32x4 res[U];
  auto tile = [&](auto uc) {
    constexpr int u = decltype(uc)::value;
    wait_vm<((U - 1 - u) * K > 63 ? 63 : (U - 1 - u) * K)>();
    asm volatile("" ::: "memory");
    f32x4 a = lds[wave][u][0][lane];
#pragma unroll
    for (int j = 1; j < K; ++j) a += lds[wave][u][j][lane];
    if constexpr (BURST) res[u] = a;
    else st_pol<ST>(dst + base + u * 64 + lane, a);
  };
  [&]<int... J>(std::integer_sequence<int, J...>) { (tile(std::integral_constant<int, J>{}), ...); }
  (std::make_integer_sequence<int, U>{});
  if constexpr (BURST) {
#pragma unroll
    for (int u = 0; u < U; ++u) st_pol<ST>(dst + base + u * 64 + lane, res[u]);
  }
}

struct Var {
  std::string name;  // a name starting "RO" moves k x n x 4 bytes (no destination)
  int threads;
  size_t per_block;  // vectors per block (one-shot); 0 = persistent
  int blocks_p;      // persistent grid
  void (*launch)(const void* const*, void*, size_t, dim3, dim3, hipStream_t);
};

template <int K, class F>
void fill_srcs(Srcs<K>& s, const void* const* p) {
  for (int j = 0; j < K; ++j) s.p[j] = static_cast<const f32x4*>(p[j]);
}

template <int K, int U, int W = 4>
void L_lds(const void* const* p, void* d, size_t nvec, dim3 g, dim3 b, hipStream_t s) {
  Srcs<K> a;
  for (int j = 0; j < K; ++j) a.p[j] = static_cast<const f32x4*>(p[j]);
  hipLaunchKernelGGL((k_lds<K, U, W>), g, b, 0, s, a, static_cast<f32x4*>(d), nvec);
}
template <int K, int U, int W, int SW = 0, bool RO = false, int ST = 0, int ORD = 0, bool BURST = false>
void L_prog(const void* const* p, void* d, size_t nvec, dim3 g, dim3 b, hipStream_t s) {
  Srcs<K> a;
  for (int j = 0; j < K; ++j) a.p[j] = static_cast<const f32x4*>(p[j]);
  hipLaunchKernelGGL((k_prog<K, U, W, SW, RO, ST, ORD, BURST>), g, b, 0, s, a, static_cast<f32x4*>(d), nvec);
}
template <int K, int U, int D, int W>
void L_ring(const void* const* p, void* d, size_t nvec, dim3 g, dim3 b, hipStream_t s) {
  Srcs<K> a;
  for (int j = 0; j < K; ++j) a.p[j] = static_cast<const f32x4*>(p[j]);
  hipLaunchKernelGGL((k_ring<K, U, D, W>), g, b, 0, s, a, static_cast<f32x4*>(d), nvec);
}
template <int K, int U, int D, int W>
void L_ringp(const void* const* p, void* d, size_t nvec, dim3 g, dim3 b, hipStream_t s) {
  Srcs<K> a;
  for (int j = 0; j < K; ++j) a.p[j] = static_cast<const f32x4*>(p[j]);
  hipLaunchKernelGGL((k_ring_p<K, U, D, W>), g, b, 0, s, a, static_cast<f32x4*>(d), nvec);
}
template <int K, int U, int W>
void L_reg(const void* const* p, void* d, size_t nvec, dim3 g, dim3 b, hipStream_t s) {
  Srcs<K> a;
  for (int j = 0; j < K; ++j) a.p[j] = static_cast<const f32x4*>(p[j]);
  hipLaunchKernelGGL((k_reg<K, U, W>), g, b, 0, s, a, static_cast<f32x4*>(d), nvec);
}

template <int K>
std::vector<Var> variants() {
  std::vector<Var> v;
  v.push_back({"prog U4 W2 (production k8)", 128, 2 * 4 * 64, 0, L_prog<K, 4, 2>});
  v.push_back({"prog U4 W2, 2 regions", 128, 2 * 4 * 64, 0, L_prog<K, 4, 2, 3>});
  v.push_back({"prog U4 W2, 4 regions", 128, 2 * 4 * 64, 0, L_prog<K, 4, 2, 4>});
  v.push_back({"prog U4 W2, 8 regions", 128, 2 * 4 * 64, 0, L_prog<K, 4, 2, 5>});
  v.push_back({"prog U1 W2 (production k2)", 128, 2 * 1 * 64, 0, L_prog<K, 1, 2>});
  v.push_back({"prog U1 W2, 2 regions", 128, 2 * 1 * 64, 0, L_prog<K, 1, 2, 3>});
  v.push_back({"prog U1 W2, 4 regions", 128, 2 * 1 * 64, 0, L_prog<K, 1, 2, 4>});
  v.push_back({"prog U1 W2, 8 regions", 128, 2 * 1 * 64, 0, L_prog<K, 1, 2, 5>});
  // one-wave workgroups: LDS per WG = U x K KiB, so up to 160 / (U K) workgroups per CU
  v.push_back({"prog U2 W1", 64, 1 * 2 * 64, 0, L_prog<K, 2, 1>});
  v.push_back({"prog U1 W1", 64, 1 * 1 * 64, 0, L_prog<K, 1, 1>});
  v.push_back({"prog U3 W1", 64, 1 * 3 * 64, 0, L_prog<K, 3, 1>});
  v.push_back({"prog U2 W1 burst", 64, 1 * 2 * 64, 0, L_prog<K, 2, 1, 0, false, 0, 0, true>});
  v.push_back({"prog U2 W1 plain st", 64, 1 * 2 * 64, 0, L_prog<K, 2, 1, 0, false, 1>});
  v.push_back({"prog U1 W2", 128, 2 * 1 * 64, 0, L_prog<K, 1, 2>});
  v.push_back({"prog U4 W4", 256, 4 * 4 * 64, 0, L_prog<K, 4, 4>});
  return v;
}

int main(int argc, char** argv) {
  const int k = argc > 1 ? atoi(argv[1]) : 8;
  const size_t n = argc > 2 ? strtoull(argv[2], nullptr, 0) : (size_t)1 << 26;
  const int sets = argc > 3 ? atoi(argv[3]) : 4;
  const int reps = argc > 4 ? atoi(argv[4]) : 8;
  const int rounds = argc > 5 ? atoi(argv[5]) : 5;
  const size_t delta = argc > 6 ? strtoull(argv[6], nullptr, 0) : 0;
  const int only = argc > 7 ? atoi(argv[7]) : -1;  // run only variants [0, only)
  const size_t nvec = n / 4;
  std::vector<Var> vars = k == 9 ? variants<9>() : k == 8 ? variants<8>() : k == 4 ? variants<4>() : k == 3 ? variants<3>() : variants<2>();
  if (only > 0 && (size_t)only < vars.size()) vars.resize(only);
  // buffers: sets x (k sources + 1 dst) + a reference output
  // one allocation per set; buffer i of a set starts at i * (n*4 + delta) (delta in bytes, a
  // multiple of 16): moves the streams' relative placement over HBM channels and banks
  std::vector<std::vector<void*>> buf(sets, std::vector<void*>(k + 1));
  for (auto& s : buf) {
    char* base;
    CHECK(hipMalloc((void**)&base, (k + 1) * (n * 4 + delta)));
    for (int i = 0; i <= k; ++i) s[i] = base + i * (n * 4 + delta);
  }
  void* ref;
  CHECK(hipMalloc(&ref, n * 4));
  {
    std::vector<float> h(n);
    unsigned long long x = 0x5EED;
    for (int si = 0; si < sets; ++si)
      for (int j = 0; j < k; ++j) {
        for (size_t i = 0; i < n; ++i) {
          x += 0x9E3779B97F4A7C15ull;
          unsigned long long z = x;
          z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
          z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
          z ^= z >> 31;
          h[i] = (float)((z >> 40) * (1.0 / 16777216.0)) * 2.f - 1.f;
        }
        CHECK(hipMemcpy(buf[si][j], h.data(), n * 4, hipMemcpyHostToDevice));
      }
  }
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto launch = [&](const Var& v, int si, void* dst) {
    const dim3 b(v.threads);
    const dim3 g(v.per_block ? (unsigned)((nvec + v.per_block - 1) / v.per_block) : (unsigned)v.blocks_p);
    v.launch(buf[si].data(), dst, nvec, g, b, st);
  };
  // correctness: set 0 through variant 0 = reference, then every variant vs it
  launch(vars[0], 0, ref);
  CHECK(hipStreamSynchronize(st));
  std::vector<unsigned> hr(n), hv(n);
  CHECK(hipMemcpy(hr.data(), ref, n * 4, hipMemcpyDeviceToHost));
  std::vector<bool> ok(vars.size(), true);
  for (size_t vi = 0; vi < vars.size(); ++vi) {
    CHECK(hipMemset(buf[0][k], 0xff, n * 4));
    launch(vars[vi], 0, buf[0][k]);
    CHECK(hipStreamSynchronize(st));
    CHECK(hipGetLastError());
    CHECK(hipMemcpy(hv.data(), buf[0][k], n * 4, hipMemcpyDeviceToHost));
    ok[vi] = vars[vi].name.rfind("RO", 0) == 0 || memcmp(hr.data(), hv.data(), n * 4) == 0;
    if (!ok[vi]) {
      size_t bad = 0;
      while (bad < n && hr[bad] == hv[bad]) ++bad;
      printf("MISMATCH %s at %zu\n", vars[vi].name.c_str(), bad);
    }
  }
  std::vector<std::vector<float>> ms(vars.size());
  for (int r = 0; r < rounds; ++r)
    for (size_t vi = 0; vi < vars.size(); ++vi) {
      for (int si = 0; si < sets; ++si) launch(vars[vi], si, buf[si][k]);  // warm the code, cold the data
      CHECK(hipEventRecord(e0, st));
      for (int i = 0; i < reps; ++i) launch(vars[vi], i % sets, buf[i % sets][k]);
      CHECK(hipEventRecord(e1, st));
      CHECK(hipEventSynchronize(e1));
      float t;
      CHECK(hipEventElapsedTime(&t, e0, e1));
      ms[vi].push_back(t / reps);
    }
  for (size_t vi = 0; vi < vars.size(); ++vi) {
    const double bytes = (double)(vars[vi].name.rfind("RO", 0) == 0 ? k : k + 1) * n * 4;
    auto m = ms[vi];
    std::sort(m.begin(), m.end());
    const double med = m[m.size() / 2];
    printf("{\"delta\": %zu, \"k\": %d, \"sets\": %d, \"variant\": \"%s\", \"ok\": %s, \"us_med\": %.2f, \"GBps_med\": %.1f, \"GBps_max\": %.1f}\n", delta, k,
           sets, vars[vi].name.c_str(), ok[vi] ? "true" : "false", med * 1e3, bytes / med / 1e6, bytes / m[0] / 1e6);
  }
  return 0;
}
