// k-way element-wise reduce for gfx950 (MI355X).
//
// Replaces FlexTree::reduce_sum<T>/reduce_band<T> (allreduce_over_mpi/mpi_mod.hpp:812-1251)
// and the reference's never-wired GPU twin reduce_sum_1..20 (vector_add/reduce_sum_gpu.h:4-316).
//
//   dst[i] = src0[i] OP src1[i] OP ... OP src{k-1}[i]      strictly left to right
//
// Design (bandwidth-bound: (k+1)*n*sizeof(T) bytes, ~0 flops per byte, no MFMA):
//   * 16 B per lane per access, one wave instruction = 1 KiB contiguous per
//     source: fully coalesced;
//   * k = 2..16 for fp32/bf16, k = 2..8 for the other types: reduce_lds_kernel stages
//     U tiles of every source per wave through LDS with LDS-DMA
//     (global_load_lds_dwordx4, nontemporal) and folds tile by tile as each
//     tile lands (counted vmcnt); stores are nontemporal too (cold data: every
//     piece of an AllReduce is new); (U, waves per workgroup) per k below;
//   * other k / types: reduce_vec_kernel, registers, 2 vectors of every source
//     per lane in flight, runtime k up to FTAR_MAX_K;
//   * one-shot grids (>> 256 CUs); source pointers travel in the kernarg
//     segment (no device-side pointer table);
//   * unaligned heads/tails (block offsets need not be 16-B aligned) are done
//     element-wise by workgroup 0 in the same launch; sources whose alignment
//     differs from dst's take an element-wise kernel instead;
//   * dst may alias a source (the ring folds in place, mpi_mod.hpp:1699):
//     every lane loads its element of every source before it stores that
//     element, so no pointer is declared __restrict__;
//   * arithmetic follows the reference's C++ semantics bit for bit:
//       float/double in their own precision (no FMA: pure adds),
//       narrow integers wrap (promotion + truncating store == modular add),
//       bool sum = OR of non-zero, bf16 (extension) = fp32 accumulate + one RNE.
#pragma once
// Internal: the reduce kernels, their traits and launchers, included by reduce_kernels.hip (the
// production dispatch, libftar.so) and bench_kernels.hip (the A/B harness, libftar_bench.so);
// anonymous namespace: each TU instantiates what it uses.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <initializer_list>
#include <type_traits>
#include <utility>

#include "ftar_internal.h"

namespace ftar {

// The kernel the launchers below launched last on this thread (its host-side handle):
// ftar_debug_last_kernel names it, so bench.py reports PMC traffic only for the kernel it timed.
inline thread_local const void* g_last_kernel = nullptr;
#define FTAR_LAUNCH(KERNEL, ...)                                         \
  do {                                                                   \
    ::ftar::g_last_kernel = reinterpret_cast<const void*>(KERNEL);       \
    hipLaunchKernelGGL(KERNEL, __VA_ARGS__);                             \
  } while (0)

namespace {

constexpr int kThreads = 256;
constexpr int kTreeLevels = kMaxFoldLevels;
// Measured on MI355X with COLD data (tools/kbench_cold.py: launches rotate over
// 4 disjoint buffer sets, so nothing is left in the 256 MB Infinity Cache from
// the previous launch -- the AllReduce's situation, where every piece is new
// data; DESIGN.md §3, profiles/r01/kbench_cold*.log):
//  * nontemporal loads AND stores (f32 k = 2: 6.55 TB/s vs 6.09 with plain
//    stores; rewriting the same destination back to back -- the reference
//    harness's loop -- favours plain stores instead, because the MALL absorbs
//    part of the writes, a regime the hot path never sees);
//  * k = 2..16: staged through LDS (LDS-DMA, no VGPR landing zone) -- f32
//    +1 % at k = 2 and +3-5 % at k = 4..8 over the best register variant
//    (round 1); folding each tile as it lands instead of after all K x U
//    loads: +0.5-2 % for f32, up to +8 % for bf16 at k = 8 (round 2);
//  * larger k (runtime k): registers, 2 vectors per lane, 512-thread workgroups.
constexpr int kUnroll = 2;
constexpr int kVecThreads = 512;
constexpr bool kNtLoads = true, kNtStores = true;
#ifndef KHW_BF16_DEFAULT
#define KHW_BF16_DEFAULT true
#endif
#ifndef KLDS_DEEP_BF16
#define KLDS_DEEP_BF16 true
#endif
// Tiles per wave (U) and waves per workgroup (W) of the LDS-staged kernel by
// element size and k, from a cold-data sweep of 14 (U, W) shapes x k = 2..16
// x {f32, bf16} on MI355X (tools/kbench_cold.py variants 40-53,
// profiles/r02/kbench_cold_prog_shapes.log).  Up to k = 4 deep per-wave
// queues win (U = 3-4); from k = 5 on, two workgroups per CU of 2-6 waves.
// Round 2 added one-wave and two-wave workgroups of 1-4 tiles (variants 54-59,
// profiles/r02/kbench_cold_small_wg.log, kbench_k2_shape_ab.log): for 4-byte
// k = 2, U = 1 x W = 2 (4 KiB of LDS, up to 16 workgroups per CU) measured
// +0.6 / +1.3 / +1.8 % over U = 4 x W = 4 in three runs; elsewhere the table held.
template <class Tr, int K>
constexpr int kLdsTiles = sizeof(typename Tr::S) >= 4 ? (K == 2 ? 1 : K <= 4 ? 3 : K <= 6 ? 2 : K <= 10 ? 4 : 2)
                                                     : (K <= 4 ? 4 : K == 5 ? 2 : K == 6 ? 5 : K <= 10 ? 4 : 2);
template <class Tr, int K>
constexpr int kLdsWaves = sizeof(typename Tr::S) >= 4 ? (K == 2 ? 2 : K <= 6 ? 6 : K <= 10 ? 2 : 4)
                                                     : (K <= 4 ? 4 : K == 5 ? 5 : K <= 10 ? 2 : 4);
// LDS per workgroup = W waves x K x U x 1 KiB (<= 160 KiB): k = 16 at U = 2 stages 128 KiB

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const u32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st16(u32x4* p, u32x4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

__device__ __forceinline__ float bf16_to_f32(unsigned short h) { return __uint_as_float((unsigned)h << 16); }
// RNE to bf16; NaN stays NaN (quieted, sign and top payload kept).  Written as
// a select, not an early return: a per-element NaN branch compiles to exec-mask
// save/restore around every conversion.
__device__ __forceinline__ unsigned bf16_round_bits(float f) {  // result in the high half
  const unsigned u = __float_as_uint(f);
  const unsigned rne = u + 0x7fffu + ((u >> 16) & 1u);
  return ((u & 0x7fffffffu) > 0x7f800000u ? (u | 0x00400000u) : rne) & 0xffff0000u;
}
__device__ __forceinline__ unsigned short f32_to_bf16(float f) { return (unsigned short)(bf16_round_bits(f) >> 16); }

// ---------------------------------------------------------------------------
// element traits: scalar (S*) and 16-byte vector (V*) forms of one (dtype, op)
// ---------------------------------------------------------------------------
struct F32Sum {
  using S = float;
  using SA = float;
  using VA = f32x4;
  __device__ static SA s_init(S x) { return x; }
  __device__ static SA s_comb(SA a, S x) { return a + x; }
  __device__ static S s_fin(SA a) { return a; }
  __device__ static VA v_init(u32x4 x) { return __builtin_bit_cast(f32x4, x); }
  __device__ static VA v_comb(VA a, u32x4 x) { return a + __builtin_bit_cast(f32x4, x); }
  __device__ static u32x4 v_fin(VA a) { return __builtin_bit_cast(u32x4, a); }
  __device__ static SA s_add(SA a, SA b) { return a + b; }
  __device__ static SA s_rnd(SA a) { return a; }
  __device__ static VA v_add(VA a, VA b) { return a + b; }
  __device__ static VA v_rnd(VA a) { return a; }
};
struct F64Sum {
  using S = double;
  using SA = double;
  using VA = f64x2;
  __device__ static SA s_init(S x) { return x; }
  __device__ static SA s_comb(SA a, S x) { return a + x; }
  __device__ static S s_fin(SA a) { return a; }
  __device__ static VA v_init(u32x4 x) { return __builtin_bit_cast(f64x2, x); }
  __device__ static VA v_comb(VA a, u32x4 x) { return a + __builtin_bit_cast(f64x2, x); }
  __device__ static u32x4 v_fin(VA a) { return __builtin_bit_cast(u32x4, a); }
  __device__ static SA s_add(SA a, SA b) { return a + b; }
  __device__ static SA s_rnd(SA a) { return a; }
  __device__ static VA v_add(VA a, VA b) { return a + b; }
  __device__ static VA v_rnd(VA a) { return a; }
};
// bf16 rounding of two floats at once.  HW: gfx950's v_cvt_pk_bf16_f32 (RNE); every one of the 2^32
// float bit patterns converts to the same bf16 bits as bf16_round_bits, NaNs included
// (ftar_debug_bf16_cvt_check, tests/test_gpu_reduce.py), so the two are interchangeable.
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
template <bool HW>
__device__ __forceinline__ unsigned pack_bf16(float lo, float hi) {
  if constexpr (HW) return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{lo, hi}, bf16x2));
  else return (bf16_round_bits(lo) >> 16) | bf16_round_bits(hi);
}
template <bool HW>
struct BF16SumT {
  using S = unsigned short;
  using SA = float;
  struct VA {
    f32x4 lo, hi;
  };
  __device__ static SA s_init(S x) { return bf16_to_f32(x); }
  __device__ static SA s_comb(SA a, S x) { return a + bf16_to_f32(x); }
  __device__ static S s_fin(SA a) { return f32_to_bf16(a); }
  __device__ static f32x4 unpack(unsigned a, unsigned b) {
    f32x4 r;
    r.x = __uint_as_float(a << 16);
    r.y = __uint_as_float(a & 0xffff0000u);
    r.z = __uint_as_float(b << 16);
    r.w = __uint_as_float(b & 0xffff0000u);
    return r;
  }
  __device__ static VA v_init(u32x4 x) { return {unpack(x.x, x.y), unpack(x.z, x.w)}; }
  __device__ static VA v_comb(VA a, u32x4 x) {
    VA b = v_init(x);
    return {a.lo + b.lo, a.hi + b.hi};
  }
  __device__ static unsigned pack(float lo, float hi) { return pack_bf16<HW>(lo, hi); }
  __device__ static u32x4 v_fin(VA a) {
    return u32x4{pack(a.lo.x, a.lo.y), pack(a.lo.z, a.lo.w), pack(a.hi.x, a.hi.y), pack(a.hi.z, a.hi.w)};
  }
  // nested folds: an inner node's value is stored as bf16 by the staged
  // schedule, so it is rounded before its parent adds it
  __device__ static float rnd(float f) { return __uint_as_float(bf16_round_bits(f)); }
  __device__ static f32x4 rnd4(f32x4 v) {
    if constexpr (HW) return unpack(pack(v.x, v.y), pack(v.z, v.w));
    else return f32x4{rnd(v.x), rnd(v.y), rnd(v.z), rnd(v.w)};
  }
  __device__ static SA s_add(SA a, SA b) { return a + b; }
  __device__ static SA s_rnd(SA a) { return rnd(a); }
  __device__ static VA v_add(VA a, VA b) { return {a.lo + b.lo, a.hi + b.hi}; }
  __device__ static VA v_rnd(VA a) { return {rnd4(a.lo), rnd4(a.hi)}; }
};
// bf16 folded hop by hop: every add rounds to bf16 (the one-round ring fold has
// to reproduce the staged ring, which rounds once per hop)
template <bool HW>
struct BF16SumHopT : BF16SumT<HW> {
  using B = BF16SumT<HW>;
  using typename B::S;
  using typename B::SA;
  using typename B::VA;
  __device__ static SA s_comb(SA a, S x) { return B::rnd(a + bf16_to_f32(x)); }
  __device__ static VA v_comb(VA a, u32x4 x) {
    VA b = B::v_init(x);
    const f32x4 lo = a.lo + b.lo, hi = a.hi + b.hi;
    return {B::rnd4(lo), B::rnd4(hi)};
  }
};
constexpr bool kHwBf16 = KHW_BF16_DEFAULT;
// bf16 nested folds of three and four levels (2,2,2), (2,2,2,2) on the LDS-staged kernel: with the
// integer RNE their per-level rounds made them ALU-bound there (round 2: -2 to -25 %); with
// v_cvt_pk_bf16_f32 rounding they gain +6.6 % and +3.6 % over the register kernel (cold,
// profiles/r02/s4/kbench_nested_bf16_lds.log).  Runtime-coded bf16 shapes still lose there (2,3: -11 %,
// 3,3: -4 %) and keep the register kernel.
constexpr bool kLdsDeepBf16 = KLDS_DEEP_BF16;
using BF16Sum = BF16SumT<kHwBf16>;
using BF16SumHop = BF16SumHopT<kHwBf16>;
// modular integer sums on packed lanes (SWAR for 8/16-bit lanes)
template <class S_, unsigned HI>
struct SwarSum {
  using S = S_;
  using SA = S_;
  using VA = u32x4;
  __device__ static SA s_init(S x) { return x; }
  __device__ static SA s_comb(SA a, S x) { return (S)(a + x); }
  __device__ static S s_fin(SA a) { return a; }
  __device__ static VA v_init(u32x4 x) { return x; }
  __device__ static VA v_comb(VA a, u32x4 b) {
    const u32x4 lo = (a & ~HI) + (b & ~HI);  // carries stay inside each lane
    return lo ^ ((a ^ b) & HI);
  }
  __device__ static u32x4 v_fin(VA a) { return a; }
};
using U8Sum = SwarSum<unsigned char, 0x80808080u>;
using U16Sum = SwarSum<unsigned short, 0x80008000u>;
struct U32Sum {
  using S = unsigned;
  using SA = unsigned;
  using VA = u32x4;
  __device__ static SA s_init(S x) { return x; }
  __device__ static SA s_comb(SA a, S x) { return a + x; }
  __device__ static S s_fin(SA a) { return a; }
  __device__ static VA v_init(u32x4 x) { return x; }
  __device__ static VA v_comb(VA a, u32x4 x) { return a + x; }
  __device__ static u32x4 v_fin(VA a) { return a; }
};
struct U64Sum {
  using S = unsigned long long;
  using SA = unsigned long long;
  using VA = u64x2;
  __device__ static SA s_init(S x) { return x; }
  __device__ static SA s_comb(SA a, S x) { return a + x; }
  __device__ static S s_fin(SA a) { return a; }
  __device__ static VA v_init(u32x4 x) { return __builtin_bit_cast(u64x2, x); }
  __device__ static VA v_comb(VA a, u32x4 x) { return a + __builtin_bit_cast(u64x2, x); }
  __device__ static u32x4 v_fin(VA a) { return __builtin_bit_cast(u32x4, a); }
};
// bool "sum": the reference adds 0/1 ints and stores sum != 0 -> logical OR
struct BoolSum {
  using S = unsigned char;
  using SA = unsigned char;
  using VA = u32x4;
  __device__ static SA s_init(S x) { return x; }
  __device__ static SA s_comb(SA a, S x) { return a | x; }
  __device__ static S s_fin(SA a) { return a != 0; }
  __device__ static VA v_init(u32x4 x) { return x; }
  __device__ static VA v_comb(VA a, u32x4 x) { return a | x; }
  __device__ static u32x4 v_fin(VA a) {
    const u32x4 nz = ((a & 0x7f7f7f7fu) + 0x7f7f7f7fu) | a;  // bit 7 of each byte = byte != 0
    return (nz >> 7) & 0x01010101u;
  }
};
template <class S_>
struct Band {
  using S = S_;
  using SA = S_;
  using VA = u32x4;
  __device__ static SA s_init(S x) { return x; }
  __device__ static SA s_comb(SA a, S x) { return (S)(a & x); }
  __device__ static S s_fin(SA a) { return a; }
  __device__ static VA v_init(u32x4 x) { return x; }
  __device__ static VA v_comb(VA a, u32x4 x) { return a & x; }
  __device__ static u32x4 v_fin(VA a) { return a; }
};

template <int K>
struct Srcs {
  const void* p[K];
};

// ---------------------------------------------------------------------------
// vector kernel: K sources (K == 0: runtime k <= FTAR_MAX_K), U vectors per lane.
// Element range [head, head + nvec*VE) is vectorised; workgroup 0 also does the
// `head` leading and `tail` trailing elements element-wise.
// ---------------------------------------------------------------------------
template <class Tr, int K, int U, bool NTL, bool NTS, int BS = kThreads>
__global__ void __launch_bounds__(BS)
    reduce_vec_kernel(Srcs<(K > 0 ? K : FTAR_MAX_K)> src, int kr, void* dst, size_t nvec, int head,
                      int tail) {
  using S = typename Tr::S;
  constexpr int KK = K > 0 ? K : FTAR_MAX_K;
  const int k = K > 0 ? K : kr;
  constexpr int VE = 16 / sizeof(S);
  constexpr int kThreads = BS;
  const size_t tile_stride = (size_t)gridDim.x * (U * kThreads);
  size_t v0 = (size_t)blockIdx.x * (U * kThreads) + threadIdx.x;

  if (blockIdx.x == 0 && threadIdx.x < (unsigned)(head + tail)) {  // unaligned head / short tail
    const size_t e = threadIdx.x < (unsigned)head ? threadIdx.x : (size_t)head + nvec * VE + (threadIdx.x - head);
    typename Tr::SA a = Tr::s_init(static_cast<const S*>(src.p[0])[e]);
    for (int j = 1; j < k; ++j) a = Tr::s_comb(a, static_cast<const S*>(src.p[j])[e]);
    static_cast<S*>(dst)[e] = Tr::s_fin(a);
  }

  const u32x4* s0 = reinterpret_cast<const u32x4*>(static_cast<const S*>(src.p[0]) + head);
  u32x4* d = reinterpret_cast<u32x4*>(static_cast<S*>(dst) + head);
  for (; v0 + (U - 1) * kThreads < nvec; v0 += tile_stride) {  // full tiles: no per-vector guards
    typename Tr::VA acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = Tr::v_init(ld16<NTL>(s0 + v0 + u * kThreads));
    if constexpr (K > 0) {
      u32x4 x[KK > 1 ? KK - 1 : 1][U];
#pragma unroll
      for (int j = 1; j < KK; ++j) {
        const u32x4* sj = reinterpret_cast<const u32x4*>(static_cast<const S*>(src.p[j]) + head);
#pragma unroll
        for (int u = 0; u < U; ++u) x[j - 1][u] = ld16<NTL>(sj + v0 + u * kThreads);
      }
#pragma unroll
      for (int j = 1; j < KK; ++j)
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] = Tr::v_comb(acc[u], x[j - 1][u]);
    } else {
      for (int j = 1; j < k; ++j) {
        const u32x4* sj = reinterpret_cast<const u32x4*>(static_cast<const S*>(src.p[j]) + head);
        u32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = ld16<NTL>(sj + v0 + u * kThreads);
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] = Tr::v_comb(acc[u], x[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) st16<NTS>(d + v0 + u * kThreads, Tr::v_fin(acc[u]));
  }
  // the one partial tile (if any): guarded
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const size_t v = v0 + u * kThreads;
    if (v >= nvec) break;
    typename Tr::VA a = Tr::v_init(ld16<NTL>(s0 + v));
    for (int j = 1; j < k; ++j)
      a = Tr::v_comb(a, ld16<NTL>(reinterpret_cast<const u32x4*>(static_cast<const S*>(src.p[j]) + head) + v));
    st16<NTS>(d + v, Tr::v_fin(a));
  }
}

// LDS-staged reduce: the production kernel for k = 2..16 (launch_k; A/B
// variants in tools/kbench_cold.py).  Each wave streams U tiles of every
// source into LDS with LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave
// instruction, nontemporal, no VGPR destination); every lane reads its own
// 16 B back with ds_read_b128 and folds.  Nothing is shared between lanes in
// an element-wise sum, so LDS serves as the landing zone of the loads: K x U
// KiB in flight per wave without spending VGPRs on them.
//   PROG (production): the loads are issued tile-major and tile u is folded
// and stored as soon as its K loads have landed (counted vmcnt: loads return
// in order, so the stores also in the count can only make a wait longer),
// while tiles u+1.. are still in flight.  !PROG waits for all K x U loads
// first (the round-1 kernel, kept as an A/B variant).
// Workgroup 0 also does the `head` leading and `tail` trailing elements
// element-wise, as reduce_vec_kernel does.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N <= 63, "gfx9 vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// The staging and tile loop shared by the flat and the nested fold: `fold(get)`
// combines the K values get(0..K-1) of one 16-B vector slot (get(j) = source
// j's vector, from LDS or, on the partial tile, from memory), `elem(e)` folds
// element e alone (unaligned head / short tail, workgroup 0).
template <class Tr, int K, int U, int W, int AUX, bool PROG, class Fold, class Elem>
__device__ __forceinline__ void lds_staged(const Srcs<K>& src, void* dst, size_t nvec, int head, int tail, Fold fold,
                                           Elem elem) {
  static_assert(W * U * K <= 160, "LDS per workgroup = W x U x K KiB <= 160 KiB");
  using S = typename Tr::S;
  constexpr int VE = 16 / sizeof(S);
  __shared__ u32x4 lds[W][U][K][64];
  if (blockIdx.x == 0 && threadIdx.x < (unsigned)(head + tail)) {  // unaligned head / short tail
    const size_t e = threadIdx.x < (unsigned)head ? threadIdx.x : (size_t)head + nvec * VE + (threadIdx.x - head);
    static_cast<S*>(dst)[e] = elem(e);
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t base = ((size_t)blockIdx.x * W + wave) * (U * 64);
  u32x4* d = reinterpret_cast<u32x4*>(static_cast<S*>(dst) + head);
  auto sp = [&](int j) { return reinterpret_cast<const u32x4*>(static_cast<const S*>(src.p[j]) + head); };
  if (base + U * 64 <= nvec) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const u32x4* g = sp(j) + base + u * 64 + lane;
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)g,
                                         (__attribute__((address_space(3))) void*)&lds[wave][u][j][0], 16, 0, AUX);
      }
    if constexpr (!PROG) wait_vmcnt<0>();
    auto tile = [&](auto uc) {
      constexpr int u = decltype(uc)::value;
      // the K loads of tile u have landed (a count above 63 waits for more: still exact)
      if constexpr (PROG) wait_vmcnt<((U - 1 - u) * K > 63 ? 63 : (U - 1 - u) * K)>();
      st16<kNtStores>(d + base + u * 64 + lane, fold([&](int j) { return lds[wave][u][j][lane]; }));
    };
    [&]<int... I>(std::integer_sequence<int, I...>) { (tile(std::integral_constant<int, I>{}), ...); }
    (std::make_integer_sequence<int, U>{});
  } else {
    for (int u = 0; u < U; ++u) {
      const size_t v = base + u * 64 + lane;
      if (v >= nvec) break;
      st16<kNtStores>(d + v, fold([&](int j) { return ld16<kNtLoads>(sp(j) + v); }));
    }
  }
}

template <class Tr, int K, int U, int W, int AUX, bool PROG>
__global__ void __launch_bounds__(W * 64)
    reduce_lds_kernel(Srcs<K> src, void* dst, size_t nvec, int head, int tail) {
  using S = typename Tr::S;
  lds_staged<Tr, K, U, W, AUX, PROG>(
      src, dst, nvec, head, tail,
      [](auto get) {
        typename Tr::VA a = Tr::v_init(get(0));
#pragma unroll
        for (int j = 1; j < K; ++j) a = Tr::v_comb(a, get(j));
        return Tr::v_fin(a);
      },
      [&](size_t e) {
        typename Tr::SA a = Tr::s_init(static_cast<const S*>(src.p[0])[e]);
        for (int j = 1; j < K; ++j) a = Tr::s_comb(a, static_cast<const S*>(src.p[j])[e]);
        return Tr::s_fin(a);
      });
}

template <class Tr, int K, int U, int W = 4, int AUX = 2, bool PROG = true>
hipError_t launch_lds(const void* const* srcs, void* dst, size_t nvec, hipStream_t s, int head = 0, int tail = 0) {
  if constexpr (W * U * K > 160) {
    return hipErrorInvalidValue;
  } else {
    Srcs<K> a{};
    for (int j = 0; j < K; ++j) a.p[j] = srcs[j];
    const size_t per_block = (size_t)W * U * 64;
    const size_t blocks = (nvec + per_block - 1) / per_block;
    FTAR_LAUNCH((reduce_lds_kernel<Tr, K, U, W, AUX, PROG>), dim3((unsigned)(blocks ? blocks : 1)),
                       dim3(W * 64), 0, s, a, dst, nvec, head, tail);
    return hipGetLastError();
  }
}

// element-wise fallback for sources not co-aligned with dst
template <class Tr>
__global__ void __launch_bounds__(kThreads)
    reduce_elem_kernel(Srcs<FTAR_MAX_K> src, int k, void* dst, size_t n) {
  using S = typename Tr::S;
  const size_t stride = (size_t)gridDim.x * kThreads;
  for (size_t e = (size_t)blockIdx.x * kThreads + threadIdx.x; e < n; e += stride) {
    typename Tr::SA a = Tr::s_init(static_cast<const S*>(src.p[0])[e]);
    for (int j = 1; j < k; ++j) a = Tr::s_comb(a, static_cast<const S*>(src.p[j])[e]);
    static_cast<S*>(dst)[e] = Tr::s_fin(a);
  }
}

// ---------------------------------------------------------------------------
// nested-fold kernel: the one-round reduce-scatter of a multi-stage tree.
// The k sources are the P copies of one block in depth-first leaf order of the
// block's mixed-radix fold tree (schedule.cpp tree_leaves), so every inner
// node folds a run of consecutive values: level 0 folds leaves w0 at a time,
// level 1 folds those results w1 at a time, ...  Per leaf j the host packs one
// code byte (make_tree_code): bits 0-2 = how many levels complete after leaf
// j, bit 3+l = the value entering level l opens a new node.  The codes are
// uniform across the grid (kernarg, scalar branches); accumulators are indexed
// only by unrolled loop counters, so they stay in VGPRs.  Float sums only:
// integer sums and AND are associative, the flat kernel is exact for them.
// ---------------------------------------------------------------------------
struct TreeCode {
  unsigned char c[FTAR_MAX_K];
};

// Code byte of leaf j of a nested fold with bottom-up widths w[0..L): bits 0-2
// = levels completed after leaf j, bit 3+l = the value entering level l opens
// a new node (level L's bit marks the root slot, written but never read).
__host__ __device__ constexpr unsigned leaf_code(const int* w, int L, int j) {
  int prod[kTreeLevels] = {};
  int p = 1;
  for (int l = 0; l < L; ++l) {
    p *= w[l];
    prod[l] = p;
  }
  unsigned done = 0;
  while (done < (unsigned)L && (j + 1) % prod[done] == 0) ++done;
  unsigned code = done;
  if (j % w[0] == 0) code |= 1u << 3;
  for (unsigned l = 1; l <= done && l < (unsigned)L; ++l)
    if (((j + 1) / prod[l - 1] - 1) % w[l] == 0) code |= 1u << (3 + l);
  if (done == (unsigned)L && L < kTreeLevels) code |= 1u << (3 + L);
  return code;
}

// The common shapes at compile time: with the leaf codes constant after
// unrolling, every select and level branch of tree_push folds away and the
// nested fold is straight-line adds (and bf16 rounds).
template <int... W>
struct StaticShape {
  static constexpr int L = sizeof...(W);
  static constexpr int K = (W * ... * 1);
  __device__ static constexpr unsigned code(int j) {
    constexpr int w[L] = {W...};
    return leaf_code(w, L, j);
  }
};
struct RuntimeShape {};

template <class Tr, bool VEC>
struct TreeOps;
template <class Tr>
struct TreeOps<Tr, true> {
  using A = typename Tr::VA;
  __device__ static A add(A a, A b) { return Tr::v_add(a, b); }
  __device__ static A rnd(A a) { return Tr::v_rnd(a); }
};
template <class Tr>
struct TreeOps<Tr, false> {
  using A = typename Tr::SA;
  __device__ static A add(A a, A b) { return Tr::s_add(a, b); }
  __device__ static A rnd(A a) { return Tr::s_rnd(a); }
};

// push leaf values v[0..U) (one per vector slot) up the tree; on the last leaf
// v ends up holding the root
template <class O, int U>
__device__ __forceinline__ void tree_push(typename O::A (&acc)[kTreeLevels][U], typename O::A (&v)[U], unsigned code) {
  const unsigned done = code & 7u;
#pragma unroll
  for (int l = 0; l < kTreeLevels; ++l) {
    const bool fresh = (code >> (3 + l)) & 1u;
#pragma unroll
    for (int u = 0; u < U; ++u) acc[l][u] = fresh ? v[u] : O::add(acc[l][u], v[u]);
    if (done <= (unsigned)l) break;
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = O::rnd(acc[l][u]);
  }
}

template <class Tr>
__device__ __forceinline__ typename Tr::S tree_elem(const void* const* p, int k, const TreeCode& tc, size_t e) {
  using S = typename Tr::S;
  using O = TreeOps<Tr, false>;
  typename O::A acc[kTreeLevels][1], v[1];
  for (int j = 0; j < k; ++j) {
    v[0] = Tr::s_init(static_cast<const S*>(p[j])[e]);
    tree_push<O, 1>(acc, v, tc.c[j]);
  }
  return Tr::s_fin(v[0]);
}

template <class Tr, int K, int U, class Sh = RuntimeShape>
__global__ void __launch_bounds__(kThreads)
    reduce_tree_kernel(Srcs<(K > 0 ? K : FTAR_MAX_K)> src, int kr, TreeCode tc, void* dst, size_t nvec,
                       int head, int tail) {
  using S = typename Tr::S;
  using O = TreeOps<Tr, true>;
  const int k = K > 0 ? K : kr;
  constexpr int VE = 16 / sizeof(S);
  const size_t tile_stride = (size_t)gridDim.x * (U * kThreads);
  size_t v0 = (size_t)blockIdx.x * (U * kThreads) + threadIdx.x;

  if (blockIdx.x == 0 && threadIdx.x < (unsigned)(head + tail)) {
    const size_t e = threadIdx.x < (unsigned)head ? threadIdx.x : (size_t)head + nvec * VE + (threadIdx.x - head);
    static_cast<S*>(dst)[e] = tree_elem<Tr>(src.p, k, tc, e);
  }
  auto sp = [&](int j) { return reinterpret_cast<const u32x4*>(static_cast<const S*>(src.p[j]) + head); };
  u32x4* d = reinterpret_cast<u32x4*>(static_cast<S*>(dst) + head);
  for (; v0 + (U - 1) * kThreads < nvec; v0 += tile_stride) {
    typename O::A acc[kTreeLevels][U], v[U];
    if constexpr (K > 0) {  // every source in flight before the first add
      u32x4 x[K][U];
#pragma unroll
      for (int j = 0; j < K; ++j)
#pragma unroll
        for (int u = 0; u < U; ++u) x[j][u] = ld16<kNtLoads>(sp(j) + v0 + u * kThreads);
#pragma unroll
      for (int j = 0; j < K; ++j) {
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = Tr::v_init(x[j][u]);
        if constexpr (std::is_same_v<Sh, RuntimeShape>) tree_push<O, U>(acc, v, tc.c[j]);
        else tree_push<O, U>(acc, v, Sh::code(j));
      }
    } else {
      for (int j = 0; j < k; ++j) {
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = Tr::v_init(ld16<kNtLoads>(sp(j) + v0 + u * kThreads));
        tree_push<O, U>(acc, v, tc.c[j]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) st16<kNtStores>(d + v0 + u * kThreads, Tr::v_fin(v[u]));
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {  // the one partial tile (if any)
    const size_t vi = v0 + u * kThreads;
    if (vi >= nvec) break;
    typename O::A acc[kTreeLevels][1], v[1];
    for (int j = 0; j < k; ++j) {
      v[0] = Tr::v_init(ld16<kNtLoads>(sp(j) + vi));
      tree_push<O, 1>(acc, v, tc.c[j]);
    }
    d[vi] = Tr::v_fin(v[0]);
  }
}

template <class Tr>
__global__ void __launch_bounds__(kThreads)
    reduce_tree_elem_kernel(Srcs<FTAR_MAX_K> src, int k, TreeCode tc, void* dst, size_t n) {
  using S = typename Tr::S;
  const size_t stride = (size_t)gridDim.x * kThreads;
  for (size_t e = (size_t)blockIdx.x * kThreads + threadIdx.x; e < n; e += stride)
    static_cast<S*>(dst)[e] = tree_elem<Tr>(src.p, k, tc, e);
}

// The nested fold on the LDS-staged tile loop (lds_staged): the production
// path for the multi-stage trees' one-round reduce-scatter up to 16 ranks.
// Compile-time shapes (Sh = StaticShape) fold to straight-line adds; other
// shapes read the leaf codes from the kernarg.
template <class Tr, int K, int U, int W, class Sh>
__global__ void __launch_bounds__(W * 64)
    reduce_tree_lds_kernel(Srcs<K> src, TreeCode tc, void* dst, size_t nvec, int head, int tail) {
  using O = TreeOps<Tr, true>;
  lds_staged<Tr, K, U, W, 2, true>(
      src, dst, nvec, head, tail,
      [&](auto get) {
        typename O::A acc[kTreeLevels][1], v[1];
#pragma unroll
        for (int j = 0; j < K; ++j) {
          v[0] = Tr::v_init(get(j));
          if constexpr (std::is_same_v<Sh, RuntimeShape>) tree_push<O, 1>(acc, v, tc.c[j]);
          else tree_push<O, 1>(acc, v, Sh::code(j));
        }
        return Tr::v_fin(v[0]);
      },
      [&](size_t e) { return tree_elem<Tr>(src.p, K, tc, e); });
}

// ---------------------------------------------------------------------------
// multi-segment copy: the peer-direct all-gather pulls every rank's final block
// (over xGMI) into the caller's buffer in ONE launch.  Workgroup w copies
// piece w / m of segment w % m: consecutive workgroups -- the ones resident
// at the same time -- pull from different ranks, so every link streams at
// once (a grid.y = segment layout would dispatch segment 0's workgroups
// first and drive one link at a time).  16 B per lane per access when source and destination
// share their address mod 16 (always, in the all-gather: both sit at the same
// block offset of 256-B aligned buffers); bytes otherwise.
// ---------------------------------------------------------------------------
struct SegArgs {
  const char* src[FTAR_MAX_K];
  char* dst[FTAR_MAX_K];
  size_t bytes[FTAR_MAX_K];
};

template <bool NT>
__device__ __forceinline__ void gather_body(const SegArgs& a, int m) {
  const int sgi = (int)(blockIdx.x % (unsigned)m);
  const size_t bid = blockIdx.x / (unsigned)m, nb = gridDim.x / (unsigned)m;
  const char* src = a.src[sgi];
  char* dst = a.dst[sgi];
  const size_t n = a.bytes[sgi];
  const size_t tid = bid * kThreads + threadIdx.x, nthr = nb * kThreads;
  const uintptr_t ms = reinterpret_cast<uintptr_t>(src) & 15, md = reinterpret_cast<uintptr_t>(dst) & 15;
  if (ms != md) {
    for (size_t i = tid; i < n; i += nthr) dst[i] = src[i];
    return;
  }
  size_t head = ms ? 16 - ms : 0;
  if (head > n) head = n;
  const size_t nvec = (n - head) / 16, tail_at = head + nvec * 16;
  if (tid < head) dst[tid] = src[tid];
  if (tid < n - tail_at) dst[tail_at + tid] = src[tail_at + tid];
  const u32x4* s4 = reinterpret_cast<const u32x4*>(src + head);
  u32x4* d4 = reinterpret_cast<u32x4*>(dst + head);
  size_t v = bid * (2 * kThreads) + threadIdx.x;
  const size_t stride = nb * (2 * kThreads);
  for (; v + kThreads < nvec; v += stride) {  // streaming both ways (cold copy: 6.3 vs 5.5 TB/s for the DMA blit)
    const u32x4 x0 = ld16<NT>(s4 + v), x1 = ld16<NT>(s4 + v + kThreads);
    st16<NT>(d4 + v, x0);
    st16<NT>(d4 + v + kThreads, x1);
  }
  if (v < nvec) st16<NT>(d4 + v, ld16<NT>(s4 + v));
}

template <bool NT, bool REL = false>
__global__ void __launch_bounds__(kThreads) gather_kernel(SegArgs a, int m) {
  gather_body<NT>(a, m);
  if constexpr (REL) __threadfence_system();  // this workgroup's stores reach memory before it retires
}

// Diagnostic (engine_host.cpp FTAR_DEBUG_HOST_GATHER_LOG): the gather, and when every wave of
// the workgroup has issued its stores, one record of where and when it ran in host memory (fine-grained, not
// held in the GPU caches) {0x80000000 | XCD, HW_ID (CU, SIMD, queue, pipe), wall clock at start, at end}, and
// two device-scope atomics on its workgroup id's pair of words in device memory: how many times a workgroup
// with this id ran (0: never; 2: the id handed out twice) and the set of XCDs it ran on (bit x: XCD x).
template <bool NT>
__global__ void __launch_bounds__(kThreads) gather_logged_kernel(SegArgs a, int m, unsigned* host_log,
                                                                 unsigned* dev_log) {
  const unsigned t0 = (unsigned)wall_clock64();
  gather_body<NT>(a, m);
  __syncthreads();
  if (threadIdx.x == 0) {
    // s_getreg: HW_REG_XCC_ID (20) bits [3:0], HW_REG_HW_ID (4) whole
    const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (15 << 11)) & 15u;
    const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));
    const unsigned t1 = (unsigned)wall_clock64();
    unsigned* h = host_log + 4 * (size_t)blockIdx.x;
    h[0] = 0x80000000u | xcc;
    h[1] = hw;
    h[2] = t0;
    h[3] = t1;
    atomicAdd(dev_log + 2 * (size_t)blockIdx.x, 1u);
    atomicOr(dev_log + 2 * (size_t)blockIdx.x + 1, 1u << xcc);
  }
}

// ---------------------------------------------------------------------------
// host-side launch
// ---------------------------------------------------------------------------

template <class Tr, int K, int U, bool NTL, bool NTS, int BS>
hipError_t launch_cfg(const void* const* srcs, int k, void* dst, size_t nvec, int head, int tail, hipStream_t s,
                      size_t max_blocks) {
  constexpr int KK = K > 0 ? K : FTAR_MAX_K;
  Srcs<KK> a{};
  for (int j = 0; j < k; ++j) a.p[j] = srcs[j];
  const size_t per_block = (size_t)U * BS;
  size_t blocks = (nvec + per_block - 1) / per_block;
  if (blocks == 0) blocks = 1;  // head/tail only
  if (max_blocks && blocks > max_blocks) blocks = max_blocks;  // grid-stride over the rest
  if (blocks > 0x7fffffffull) blocks = 0x7fffffffull;
  FTAR_LAUNCH((reduce_vec_kernel<Tr, K, U, NTL, NTS, BS>), dim3((unsigned)blocks), dim3(BS), 0, s, a, k, dst,
                     nvec, head, tail);
  return hipGetLastError();
}

template <class Tr, int K>
hipError_t launch_k(const void* const* srcs, int k, void* dst, size_t nvec, int head, int tail, hipStream_t s) {
  if constexpr (K >= 2)
    return launch_lds<Tr, K, kLdsTiles<Tr, K>, kLdsWaves<Tr, K>>(srcs, dst, nvec, s, head, tail);
  else
    return launch_cfg<Tr, K, kUnroll, kNtLoads, kNtStores, kVecThreads>(srcs, k, dst, nvec, head, tail, s, 0);
}

// Leaf codes of a nested fold with bottom-up widths shape[0..nlevels) over k
// leaves (see reduce_tree_kernel).
bool make_tree_code(const int* shape, int nlevels, int k, TreeCode* tc) {
  if (nlevels < 1 || nlevels > kTreeLevels || k > FTAR_MAX_K) return false;
  size_t prod = 1;
  for (int l = 0; l < nlevels; ++l) {
    if (shape[l] < 1) return false;
    prod *= (size_t)shape[l];
  }
  if (prod != (size_t)k) return false;
  for (int j = 0; j < k; ++j) tc->c[j] = (unsigned char)leaf_code(shape, nlevels, j);
  return true;
}

template <class Tr, int K, int U, class Sh = RuntimeShape>
hipError_t launch_tree_k(const void* const* srcs, int k, const TreeCode& tc, void* dst, size_t nvec, int head,
                         int tail, hipStream_t s) {
  constexpr int KK = K > 0 ? K : FTAR_MAX_K;
  Srcs<KK> a{};
  for (int j = 0; j < k; ++j) a.p[j] = srcs[j];
  size_t blocks = (nvec + (size_t)U * kThreads - 1) / ((size_t)U * kThreads);
  if (blocks == 0) blocks = 1;
  if (blocks > 0x7fffffffull) blocks = 0x7fffffffull;
  FTAR_LAUNCH((reduce_tree_kernel<Tr, K, U, Sh>), dim3((unsigned)blocks), dim3(kThreads), 0, s, a, k, tc, dst,
                     nvec, head, tail);
  return hipGetLastError();
}

template <class Tr, int K, class Sh = RuntimeShape>
hipError_t launch_tree_lds(const void* const* srcs, const TreeCode& tc, void* dst, size_t nvec, int head, int tail,
                           hipStream_t s) {
  constexpr int U = kLdsTiles<Tr, K>, W = kLdsWaves<Tr, K>;
  Srcs<K> a{};
  for (int j = 0; j < K; ++j) a.p[j] = srcs[j];
  const size_t per_block = (size_t)W * U * 64;
  const size_t blocks = (nvec + per_block - 1) / per_block;
  FTAR_LAUNCH((reduce_tree_lds_kernel<Tr, K, U, W, Sh>), dim3((unsigned)(blocks ? blocks : 1)), dim3(W * 64),
                     0, s, a, tc, dst, nvec, head, tail);
  return hipGetLastError();
}

template <class Tr>
hipError_t launch_tree(const void* const* srcs, int k, const TreeCode& tc, const int* shape, int nlevels, void* dst,
                       size_t count, hipStream_t s, bool lds) {
  using S = typename Tr::S;
  constexpr size_t VE = 16 / sizeof(S);
  const uintptr_t mis = reinterpret_cast<uintptr_t>(dst) & 15;
  bool co_aligned = (mis % sizeof(S)) == 0;
  for (int j = 0; j < k && co_aligned; ++j) co_aligned = (reinterpret_cast<uintptr_t>(srcs[j]) & 15) == mis;
  if (!co_aligned) {
    Srcs<FTAR_MAX_K> a{};
    for (int j = 0; j < k; ++j) a.p[j] = srcs[j];
    size_t blocks = (count + kThreads - 1) / kThreads;
    blocks = blocks > 8192 ? 8192 : blocks;
    FTAR_LAUNCH((reduce_tree_elem_kernel<Tr>), dim3((unsigned)blocks), dim3(kThreads), 0, s, a, k, tc, dst,
                       count);
    return hipGetLastError();
  }
  size_t head = mis ? (16 - mis) / sizeof(S) : 0;
  if (head > count) head = count;
  const size_t nvec = (count - head) / VE;
  const int tail = (int)(count - head - nvec * VE);
  const int h = (int)head;
  auto is = [&](std::initializer_list<int> w) {
    return (int)w.size() == nlevels && std::equal(w.begin(), w.end(), shape);
  };
  // the multi-stage trees of 4, 8 and 16 ranks: compile-time shapes.
  // LDS-staged (production, round 2): cold A/B against the register kernel
  // (profiles/r02/kbench_cold_nested_lds.log): fp32 +4 to +10 % on every
  // shape; bf16 +4 to +8 % on the two-level shapes, and since bf16 rounds with
  // v_cvt_pk_bf16_f32 (kLdsDeepBf16) on (2,2,2) and (2,2,2,2) too; its
  // runtime-coded folds still lose there and keep the register kernel.
  if (lds) {
    if (is({2, 2})) return launch_tree_lds<Tr, 4, StaticShape<2, 2>>(srcs, tc, dst, nvec, h, tail, s);
    if (is({2, 4})) return launch_tree_lds<Tr, 8, StaticShape<2, 4>>(srcs, tc, dst, nvec, h, tail, s);
    if (is({4, 2})) return launch_tree_lds<Tr, 8, StaticShape<4, 2>>(srcs, tc, dst, nvec, h, tail, s);
    if (is({4, 4})) return launch_tree_lds<Tr, 16, StaticShape<4, 4>>(srcs, tc, dst, nvec, h, tail, s);
  }
  if (lds && (sizeof(S) >= 4 || kLdsDeepBf16)) {
    if (is({2, 2, 2})) return launch_tree_lds<Tr, 8, StaticShape<2, 2, 2>>(srcs, tc, dst, nvec, h, tail, s);
    if (is({2, 2, 2, 2})) return launch_tree_lds<Tr, 16, StaticShape<2, 2, 2, 2>>(srcs, tc, dst, nvec, h, tail, s);
  }
  if (lds && sizeof(S) >= 4) {
    switch (k) {  // other shapes: runtime leaf codes
      case 4: return launch_tree_lds<Tr, 4>(srcs, tc, dst, nvec, h, tail, s);
      case 6: return launch_tree_lds<Tr, 6>(srcs, tc, dst, nvec, h, tail, s);
      case 8: return launch_tree_lds<Tr, 8>(srcs, tc, dst, nvec, h, tail, s);
      case 9: return launch_tree_lds<Tr, 9>(srcs, tc, dst, nvec, h, tail, s);
      case 12: return launch_tree_lds<Tr, 12>(srcs, tc, dst, nvec, h, tail, s);
      case 16: return launch_tree_lds<Tr, 16>(srcs, tc, dst, nvec, h, tail, s);
      default: break;
    }
    return launch_tree_k<Tr, 0, 2>(srcs, k, tc, dst, nvec, h, tail, s);
  }
  // registers (round 1; the A/B reference of ftar_debug_reduce_nested_lds)
  if (is({2, 2})) return launch_tree_k<Tr, 4, 2, StaticShape<2, 2>>(srcs, k, tc, dst, nvec, h, tail, s);
  if (is({2, 4})) return launch_tree_k<Tr, 8, 2, StaticShape<2, 4>>(srcs, k, tc, dst, nvec, h, tail, s);
  if (is({4, 2})) return launch_tree_k<Tr, 8, 2, StaticShape<4, 2>>(srcs, k, tc, dst, nvec, h, tail, s);
  if (is({2, 2, 2})) return launch_tree_k<Tr, 8, 2, StaticShape<2, 2, 2>>(srcs, k, tc, dst, nvec, h, tail, s);
  if (is({4, 4})) return launch_tree_k<Tr, 16, 1, StaticShape<4, 4>>(srcs, k, tc, dst, nvec, h, tail, s);
  if (is({2, 2, 2, 2})) return launch_tree_k<Tr, 16, 1, StaticShape<2, 2, 2, 2>>(srcs, k, tc, dst, nvec, h, tail, s);
  switch (k) {  // other shapes: runtime leaf codes; 16 sources fit one vector per lane
    case 4: return launch_tree_k<Tr, 4, 2>(srcs, k, tc, dst, nvec, h, tail, s);
    case 6: return launch_tree_k<Tr, 6, 2>(srcs, k, tc, dst, nvec, h, tail, s);
    case 8: return launch_tree_k<Tr, 8, 2>(srcs, k, tc, dst, nvec, h, tail, s);
    case 16: return launch_tree_k<Tr, 16, 1>(srcs, k, tc, dst, nvec, h, tail, s);
    default: return launch_tree_k<Tr, 0, 2>(srcs, k, tc, dst, nvec, h, tail, s);
  }
}

// HOT: the largest k with an unrolled LDS-staged kernel (fp32/bf16 16, the other types 8; 0 = k = 2
// only); larger k take the runtime-k register kernel.  The other types gained 4-6 % at k = 8 on the
// LDS kernel (tools/dtype_rates.py, profiles/r02/s4/dtype_rates*.log).
template <class Tr, int HOT>
hipError_t launch_tr(const void* const* srcs, int k, void* dst, size_t count, hipStream_t s) {
  using S = typename Tr::S;
  constexpr size_t VE = 16 / sizeof(S);
  const uintptr_t mis = reinterpret_cast<uintptr_t>(dst) & 15;
  bool co_aligned = (mis % sizeof(S)) == 0;
  for (int j = 0; j < k && co_aligned; ++j) co_aligned = (reinterpret_cast<uintptr_t>(srcs[j]) & 15) == mis;
  if (!co_aligned) {
    Srcs<FTAR_MAX_K> a{};
    for (int j = 0; j < k; ++j) a.p[j] = srcs[j];
    size_t blocks = (count + kThreads - 1) / kThreads;
    blocks = blocks > 8192 ? 8192 : blocks;
    FTAR_LAUNCH((reduce_elem_kernel<Tr>), dim3((unsigned)blocks), dim3(kThreads), 0, s, a, k, dst, count);
    return hipGetLastError();
  }
  size_t head = mis ? (16 - mis) / sizeof(S) : 0;
  if (head > count) head = count;
  const size_t nvec = (count - head) / VE;
  const size_t tail = count - head - nvec * VE;
  hipError_t e = hipErrorInvalidValue;
  bool done = false;
  [&]<int... I>(std::integer_sequence<int, I...>) {  // k = 2 .. max(2, HOT), unrolled
    ((k == I + 2 && (I + 2 == 2 || I + 2 <= HOT)
          ? (e = launch_k<Tr, (I + 2 <= (HOT > 2 ? HOT : 2) ? I + 2 : 2)>(srcs, k, dst, nvec, (int)head, (int)tail, s),
             done = true)
          : false),
     ...);
  }(std::make_integer_sequence<int, (HOT > 2 ? HOT : 2) - 1>{});
  if (done) return e;
  return launch_k<Tr, 0>(srcs, k, dst, nvec, (int)head, (int)tail, s);
}

}  // namespace
}  // namespace ftar
