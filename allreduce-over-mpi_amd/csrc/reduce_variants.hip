// A/B harness of the reduce kernels (tools/kbench_cold.py; not part of ftar.h): shape, cache-policy and
// dtype variants of the production kernels in reduce_impl.h, built in their own translation unit so the
// library compiles in parallel.
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

