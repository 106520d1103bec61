// libftar_bench.so: the A/B harness of the reduce kernels and kernel-level test hooks, kept OUT of the
// product library (libftar.so holds only the kernels launch_reduce / launch_tree / launch_copy /
// launch_gather dispatch).  Not part of ftar.h; loaded by tools/kbench*.py and the bf16 conversion test
// through ftar.bench_lib().  Shape, cache-policy and dtype variants of the production kernels in
// reduce_impl.h are instantiated here from the same templates; launch_gather (variant 90) and
// launch_reduce (the nested-fold A/B) are the product's own, linked from libftar.so.
#include "reduce_impl.h"

namespace ftar {

// ---------------------------------------------------------------------------
// A/B variants for tools/kbench.py (not part of ftar.h): (U, NT loads, NT
// stores, workgroup size, grid cap) for fp32 and bf16 sums, k in {2, 4, 8}.
// ---------------------------------------------------------------------------
namespace {
// progressive LDS-staged kernel: (tiles per wave U, waves per workgroup W)
template <class Tr, int K>
hipError_t variant_prog(int v, const void* const* srcs, void* dst, size_t nvec, hipStream_t s) {
  switch (v) {
    case 40: return launch_lds<Tr, K, 4, 4>(srcs, dst, nvec, s);
    case 41: return launch_lds<Tr, K, 3, 4>(srcs, dst, nvec, s);
    case 42: return launch_lds<Tr, K, 2, 4>(srcs, dst, nvec, s);
    case 43: return launch_lds<Tr, K, 4, 2>(srcs, dst, nvec, s);
    case 44: return launch_lds<Tr, K, 3, 6>(srcs, dst, nvec, s);
    case 45: return launch_lds<Tr, K, 2, 6>(srcs, dst, nvec, s);
    case 46: return launch_lds<Tr, K, 2, 8>(srcs, dst, nvec, s);
    case 47: return launch_lds<Tr, K, 1, 8>(srcs, dst, nvec, s);
    case 48: return launch_lds<Tr, K, 3, 2>(srcs, dst, nvec, s);
    case 49: return launch_lds<Tr, K, 6, 2>(srcs, dst, nvec, s);
    case 50: return launch_lds<Tr, K, 2, 2>(srcs, dst, nvec, s);
    case 51: return launch_lds<Tr, K, 1, 4>(srcs, dst, nvec, s);
    case 52: return launch_lds<Tr, K, 5, 2>(srcs, dst, nvec, s);
    case 53: return launch_lds<Tr, K, 2, 5>(srcs, dst, nvec, s);
    // small workgroups, many per CU (round 2: tools/kexp/k8_exp.hip found U1 W2 / U2 W1 ahead at k = 2..9)
    case 54: return launch_lds<Tr, K, 1, 2>(srcs, dst, nvec, s);
    case 55: return launch_lds<Tr, K, 1, 1>(srcs, dst, nvec, s);
    case 56: return launch_lds<Tr, K, 2, 1>(srcs, dst, nvec, s);
    case 57: return launch_lds<Tr, K, 1, 3>(srcs, dst, nvec, s);
    case 58: return launch_lds<Tr, K, 3, 1>(srcs, dst, nvec, s);
    case 59: return launch_lds<Tr, K, 4, 1>(srcs, dst, nvec, s);
    // load cache policy (the aux operand of global_load_lds) at the production shape: 2 = nt (production)
    case 60: return launch_lds<Tr, K, kLdsTiles<Tr, K>, kLdsWaves<Tr, K>, 1>(srcs, dst, nvec, s);
    case 61: return launch_lds<Tr, K, kLdsTiles<Tr, K>, kLdsWaves<Tr, K>, 3>(srcs, dst, nvec, s);
    case 62: return launch_lds<Tr, K, kLdsTiles<Tr, K>, kLdsWaves<Tr, K>, 2>(srcs, dst, nvec, s);
  }
  return hipErrorInvalidValue;
}
template <class Tr, int K>
hipError_t variant_k(int v, const void* const* srcs, int k, void* dst, size_t nvec, hipStream_t s) {
  switch (v) {
    case 0: return launch_cfg<Tr, K, 2, true, false, 256>(srcs, k, dst, nvec, 0, 0, s, 0);
    case 1: return launch_cfg<Tr, K, 1, true, false, 256>(srcs, k, dst, nvec, 0, 0, s, 0);
    case 2: return launch_cfg<Tr, K, 4, true, false, 256>(srcs, k, dst, nvec, 0, 0, s, 0);
    case 3: return launch_cfg<Tr, K, 1, true, false, 512>(srcs, k, dst, nvec, 0, 0, s, 0);
    case 4: return launch_cfg<Tr, K, 2, true, false, 512>(srcs, k, dst, nvec, 0, 0, s, 0);
    case 5: return launch_cfg<Tr, K, 1, true, false, 1024>(srcs, k, dst, nvec, 0, 0, s, 0);
    case 6: return launch_cfg<Tr, K, 2, true, false, 128>(srcs, k, dst, nvec, 0, 0, s, 0);
    case 7: return launch_cfg<Tr, K, 2, false, false, 256>(srcs, k, dst, nvec, 0, 0, s, 0);
    case 8: return launch_cfg<Tr, K, 1, true, false, 256>(srcs, k, dst, nvec, 0, 0, s, 2048);
    case 9: return launch_cfg<Tr, K, 2, true, false, 256>(srcs, k, dst, nvec, 0, 0, s, 4096);
    case 10: return launch_cfg<Tr, K, 1, true, false, 128>(srcs, k, dst, nvec, 0, 0, s, 0);
    case 11: return launch_cfg<Tr, K, 4, true, false, 128>(srcs, k, dst, nvec, 0, 0, s, 0);
    case 12: return launch_cfg<Tr, K, 2, true, true, 256>(srcs, k, dst, nvec, 0, 0, s, 0);   // nt stores
    case 13: return launch_cfg<Tr, K, 1, true, true, 256>(srcs, k, dst, nvec, 0, 0, s, 0);
    case 14: return launch_cfg<Tr, K, 4, true, true, 256>(srcs, k, dst, nvec, 0, 0, s, 0);
    case 15: return launch_cfg<Tr, K, 2, false, true, 256>(srcs, k, dst, nvec, 0, 0, s, 0);
    case 16: return launch_cfg<Tr, K, 2, true, true, 512>(srcs, k, dst, nvec, 0, 0, s, 0);
    case 17: return launch_cfg<Tr, K, 4, true, false, 256>(srcs, k, dst, nvec, 0, 0, s, 4096);
    case 18: return launch_cfg<Tr, K, 2, true, true, 256>(srcs, k, dst, nvec, 0, 0, s, 8192);
    case 19: return launch_cfg<Tr, K, 4, true, true, 512>(srcs, k, dst, nvec, 0, 0, s, 0);
    case 23: return launch_cfg<Tr, K, 4, true, true, 128>(srcs, k, dst, nvec, 0, 0, s, 0);
    case 24: return launch_cfg<Tr, K, 8, true, true, 256>(srcs, k, dst, nvec, 0, 0, s, 0);
    case 25: return launch_cfg<Tr, K, 2, true, true, 128>(srcs, k, dst, nvec, 0, 0, s, 0);
    case 26: return launch_cfg<Tr, K, 1, true, true, 512>(srcs, k, dst, nvec, 0, 0, s, 0);
    case 31: return launch_lds<Tr, K, (K <= 4 ? 4 : 2), 4, 2, false>(srcs, dst, nvec, s);
    case 32: return launch_lds<Tr, K, (K <= 4 ? 4 : (K <= 6 ? 3 : 2)), 4, 2, false>(srcs, dst, nvec, s);
    case 33: return launch_lds<Tr, K, 1, 4, 2, false>(srcs, dst, nvec, s);
    case 27: return launch_cfg<Tr, 0, 2, true, true, 512>(srcs, k, dst, nvec, 0, 0, s, 0);  // runtime-k loop
    case 28: return launch_cfg<Tr, 0, 4, true, true, 256>(srcs, k, dst, nvec, 0, 0, s, 0);
    case 29: return launch_cfg<Tr, 0, 1, true, true, 512>(srcs, k, dst, nvec, 0, 0, s, 0);
    case 30: return launch_cfg<Tr, 0, 2, true, true, 256>(srcs, k, dst, nvec, 0, 0, s, 0);
    case 20: return launch_lds<Tr, K, 2, 4, 2, false>(srcs, dst, nvec, s);  // LDS-DMA, nt, wait for all
    case 21: return launch_lds<Tr, K, 4, 4, 2, false>(srcs, dst, nvec, s);
    case 22: return launch_lds<Tr, K, 2, 4, 0, false>(srcs, dst, nvec, s);  // LDS-DMA, default policy
  }
  return variant_prog<Tr, K>(v, srcs, dst, nvec, s);
}
// k = 1 (a copy, vector_add/reduce_sum.h:36-47): variant 90 = production (the streaming copy kernel,
// launch_gather), 40-62 = the LDS-DMA-staged kernel with K = 1 (load to LDS, store from LDS)
template <class Tr>
hipError_t variant_copy(int v, const void* const* srcs, void* dst, size_t nvec, hipStream_t s) {
  if (v == 90) {
    const Segment seg{srcs[0], dst, nvec * 16};
    return launch_gather(&seg, 1, s) == FTAR_SUCCESS ? hipSuccess : hipErrorInvalidValue;
  }
  return variant_prog<Tr, 1>(v, srcs, dst, nvec, s);
}

template <class Tr>
hipError_t variant_tr(int v, const void* const* srcs, int k, void* dst, size_t nvec, hipStream_t s) {
  switch (k) {
    case 1: return variant_copy<Tr>(v, srcs, dst, nvec, s);
    case 2: return variant_k<Tr, 2>(v, srcs, k, dst, nvec, s);
    case 3: return variant_k<Tr, 3>(v, srcs, k, dst, nvec, s);
    case 4: return variant_k<Tr, 4>(v, srcs, k, dst, nvec, s);
    case 5: return variant_prog<Tr, 5>(v, srcs, dst, nvec, s);
    case 6: return variant_k<Tr, 6>(v, srcs, k, dst, nvec, s);
    case 7: return variant_prog<Tr, 7>(v, srcs, dst, nvec, s);
    case 8: return variant_k<Tr, 8>(v, srcs, k, dst, nvec, s);
    case 10: return variant_prog<Tr, 10>(v, srcs, dst, nvec, s);
    case 12: return variant_prog<Tr, 12>(v, srcs, dst, nvec, s);
    case 16: return variant_prog<Tr, 16>(v, srcs, dst, nvec, s);
  }
  return hipErrorInvalidValue;
}
}  // namespace

hipError_t hop_variant(int v, const void* const* srcs, int k, void* dst, size_t nvec, hipStream_t s) {
  switch (k) {
    case 2: return variant_prog<BF16SumHop, 2>(v, srcs, dst, nvec, s);
    case 4: return variant_prog<BF16SumHop, 4>(v, srcs, dst, nvec, s);
    case 8: return variant_prog<BF16SumHop, 8>(v, srcs, dst, nvec, s);
    case 16: return variant_prog<BF16SumHop, 16>(v, srcs, dst, nvec, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace ftar

extern "C" ftar_status_t ftar_debug_reduce_variant(int variant, int dtype, const void* const* srcs, int k, void* dst,
                                                   size_t count, void* stream) {
  if (reinterpret_cast<uintptr_t>(dst) & 15) return FTAR_ERR_INVALID_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipError_t e;
  if (dtype == FTAR_FLOAT32 && count % 4 == 0) e = ftar::variant_tr<ftar::F32Sum>(variant, srcs, k, dst, count / 4, s);
  else if (dtype == FTAR_BFLOAT16 && count % 8 == 0)
    e = ftar::variant_tr<ftar::BF16Sum>(variant, srcs, k, dst, count / 8, s);
  // 100 + bf16: the ring's hop fold (rounds after every add), production shape (variant 62), k = 2, 4, 8, 16.
  // (The round-2 A/B of the two bf16 conversions, profiles/r02/s4/kbench_bf16_cvt.log, also built
  // 200 + bf16 / 300 + bf16 for the flat and hop folds with the integer RNE; dropped to keep build time.)
  else if (dtype == 100 + FTAR_BFLOAT16 && count % 8 == 0)
    e = ftar::hop_variant(variant, srcs, k, dst, count / 8, s);
  else return FTAR_ERR_INVALID_ARG;
  return e == hipSuccess ? FTAR_SUCCESS : FTAR_ERR_HIP;
}

// A/B of the nested fold: lds = 1 the LDS-staged kernel (production), 0 the
// register kernel of round 1 (tools/kbench_cold.py --shapes).
extern "C" ftar_status_t ftar_debug_reduce_nested_lds(int lds, const void* const* srcs, int k, void* dst, size_t count,
                                                      int dtype, const int* shape, int nlevels, void* stream) {
  return ftar::launch_reduce(srcs, k, dst, count, (ftar_dtype_t)dtype, FTAR_SUM, static_cast<hipStream_t>(stream),
                             false, shape, nlevels, lds != 0);
}

namespace ftar {
namespace {
// every float bit pattern u (lo half) and u ^ 0x80000001 (hi half) through both bf16 conversions
__global__ void __launch_bounds__(256) bf16_cvt_check_kernel(unsigned long long* bad, unsigned* first) {
  const unsigned long long stride = (unsigned long long)gridDim.x * 256;
  unsigned long long mine = 0;
  unsigned first_mine = 0xffffffffu;
  for (unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x; i < (1ull << 32); i += stride) {
    const unsigned u = (unsigned)i, v = u ^ 0x80000001u;
    const float lo = __uint_as_float(u), hi = __uint_as_float(v);
    if (pack_bf16<true>(lo, hi) != pack_bf16<false>(lo, hi)) {
      ++mine;
      first_mine = first_mine < u ? first_mine : u;
    }
  }
  if (mine) {
    atomicAdd(bad, mine);
    atomicMin(first, first_mine);
  }
}
}  // namespace
}  // namespace ftar

// Test hook (not in ftar.h): how many of the 2^32 float bit patterns convert to different bf16 bits
// through v_cvt_pk_bf16_f32 than through the bit-exact RNE (bf16_round_bits); the first such pattern.
extern "C" ftar_status_t ftar_debug_bf16_cvt_check(unsigned long long* mismatches, unsigned* first) {
  if (!mismatches || !first) return FTAR_ERR_INVALID_ARG;
  unsigned long long* d_bad = nullptr;
  unsigned* d_first = nullptr;
  ftar_status_t st = FTAR_SUCCESS;  // both buffers are freed on every path below
  if (hipMalloc(&d_bad, sizeof *d_bad) != hipSuccess || hipMalloc(&d_first, sizeof *d_first) != hipSuccess)
    st = FTAR_ERR_NO_MEMORY;
  if (st == FTAR_SUCCESS &&
      (hipMemset(d_bad, 0, sizeof *d_bad) != hipSuccess || hipMemset(d_first, 0xff, sizeof *d_first) != hipSuccess))
    st = FTAR_ERR_HIP;
  if (st == FTAR_SUCCESS) {
    hipLaunchKernelGGL(ftar::bf16_cvt_check_kernel, dim3(8192), dim3(256), 0, nullptr, d_bad, d_first);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(mismatches, d_bad, sizeof *d_bad, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(first, d_first, sizeof *d_first, hipMemcpyDeviceToHost) != hipSuccess)
      st = FTAR_ERR_HIP;
  }
  ftar::hip_ignore(hipFree(d_bad));
  ftar::hip_ignore(hipFree(d_first));
  return st;
}

// ---------------------------------------------------------------------------
// Rehearsal hook of bench.py: a stream that really never drains while the RCCL preflight is
// waited for.  One wave spins on a host flag (a system-scope atomic load, vector memory) until the host
// releases it or `seconds` pass -- every wave reaches that exit, so the stream always drains in the end.
// ---------------------------------------------------------------------------
namespace {
__global__ void block_stream_kernel(int* flag, unsigned long long limit_ticks) {
  const unsigned long long t0 = wall_clock64();
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0 &&
         wall_clock64() - t0 < limit_ticks)
    __builtin_amdgcn_s_sleep(8);
}
}  // namespace

// Enqueues the spinning wave on `stream`; returns the host flag to release (ftar_debug_unblock), or NULL.
extern "C" void* ftar_debug_block_stream(void* stream, double seconds) {
  int* flag = nullptr;
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&flag), sizeof(int), hipHostMallocCoherent | hipHostMallocMapped) !=
          hipSuccess)
    return nullptr;
  __atomic_store_n(flag, 0, __ATOMIC_SEQ_CST);
  const unsigned long long ticks = (unsigned long long)(seconds * 1e3 * khz);
  hipLaunchKernelGGL(block_stream_kernel, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream), flag, ticks);
  if (hipGetLastError() != hipSuccess) return nullptr;
  return flag;
}

// Releases a stream blocked by ftar_debug_block_stream (the 4-byte flag stays allocated).
extern "C" void ftar_debug_unblock(void* flag) {
  if (flag) __atomic_store_n(static_cast<int*>(flag), 1, __ATOMIC_SEQ_CST);
}
