// Production dispatch of the k-way reduce (ftar_reduce, the engine's folds) and the streaming copy;
// kernels and traits in reduce_impl.h.  Replaces FlexTree::reduce_sum<T>/reduce_band<T>
// (allreduce_over_mpi/mpi_mod.hpp:812-1251) and reduce_sum_gpu (vector_add/reduce_sum_gpu.h:205).
#include "reduce_impl.h"

#include <cxxabi.h>

#include <cstdlib>
#include <cstring>

namespace ftar {

size_t dtype_size(ftar_dtype_t dt) {
  switch (dt) {
    case FTAR_UINT8: case FTAR_INT8: case FTAR_BOOL: return 1;
    case FTAR_UINT16: case FTAR_INT16: case FTAR_BFLOAT16: return 2;
    case FTAR_INT32: case FTAR_FLOAT32: return 4;
    case FTAR_INT64: case FTAR_FLOAT64: return 8;
  }
  return 0;
}

bool dtype_op_supported(ftar_dtype_t dt, ftar_op_t op) {
  if (dtype_size(dt) == 0) return false;
  if (op == FTAR_SUM) return true;
  if (op == FTAR_BAND)  // mpi_mod.hpp:1389-1396: integer types only
    return dt == FTAR_UINT8 || dt == FTAR_INT8 || dt == FTAR_UINT16 || dt == FTAR_INT16 || dt == FTAR_INT32 ||
           dt == FTAR_INT64;
  return false;
}

namespace {
// the segments with bytes, packed, and the grid: workgroups per segment to cover the largest in one pass
// (at most 65535, then grid-stride; max_wg_per_seg caps it), times the segments
GatherGeom pack_segments(const Segment* segs, int nsegs, size_t max_wg_per_seg, SegArgs* a) {
  GatherGeom g;
  size_t most = 0;
  for (int i = 0; i < nsegs; ++i) {
    if (!segs[i].bytes) continue;
    a->src[g.nsegs] = static_cast<const char*>(segs[i].src);
    a->dst[g.nsegs] = static_cast<char*>(segs[i].dst);
    a->bytes[g.nsegs] = segs[i].bytes;
    most = std::max(most, segs[i].bytes);
    ++g.nsegs;
  }
  if (!g.nsegs) return g;
  size_t bx = (most / 16 + 2 * kThreads - 1) / (2 * kThreads);
  bx = std::max<size_t>(1, std::min<size_t>(bx, 65535));  // per segment; grid-stride beyond
  if (max_wg_per_seg) bx = std::min(bx, max_wg_per_seg);
  g.grid = (unsigned)(bx * (size_t)g.nsegs);
  g.tile_bytes = 2 * kThreads * 16;
  return g;
}
}  // namespace

GatherGeom gather_geometry(const Segment* segs, int nsegs, size_t max_wg_per_seg) {
  if (nsegs < 0 || nsegs > FTAR_MAX_K) return GatherGeom{};
  SegArgs a{};
  return pack_segments(segs, nsegs, max_wg_per_seg, &a);
}

ftar_status_t launch_gather(const Segment* segs, int nsegs, hipStream_t stream, bool nt, size_t max_wg_per_seg,
                            bool release_system) {
  if (nsegs < 0 || nsegs > FTAR_MAX_K) return FTAR_ERR_INVALID_ARG;
  SegArgs a{};
  const GatherGeom g = pack_segments(segs, nsegs, max_wg_per_seg, &a);
  if (!g.nsegs) return FTAR_SUCCESS;
  const int m = (int)g.nsegs;
  const dim3 grid(g.grid);
  if (release_system && nt)
    FTAR_LAUNCH((gather_kernel<true, true>), grid, dim3(kThreads), 0, stream, a, m);
  else if (release_system)
    FTAR_LAUNCH((gather_kernel<false, true>), grid, dim3(kThreads), 0, stream, a, m);
  else if (nt)
    FTAR_LAUNCH(gather_kernel<true>, grid, dim3(kThreads), 0, stream, a, m);
  else
    FTAR_LAUNCH(gather_kernel<false>, grid, dim3(kThreads), 0, stream, a, m);
  FTAR_CHECK_HIP(hipGetLastError());
  return FTAR_SUCCESS;
}

ftar_status_t launch_gather_logged(const Segment* segs, int nsegs, hipStream_t stream, bool nt,
                                   size_t max_wg_per_seg, unsigned* host_log, unsigned* dev_log, size_t cap_wg) {
  if (nsegs < 0 || nsegs > FTAR_MAX_K || !host_log || !dev_log) return FTAR_ERR_INVALID_ARG;
  SegArgs a{};
  const GatherGeom g = pack_segments(segs, nsegs, max_wg_per_seg, &a);
  if (!g.nsegs) return FTAR_SUCCESS;
  if (g.grid > cap_wg) return FTAR_ERR_INVALID_ARG;  // one record per workgroup must fit
  const int m = (int)g.nsegs;
  if (nt)
    FTAR_LAUNCH(gather_logged_kernel<true>, dim3(g.grid), dim3(kThreads), 0, stream, a, m, host_log, dev_log);
  else
    FTAR_LAUNCH(gather_logged_kernel<false>, dim3(g.grid), dim3(kThreads), 0, stream, a, m, host_log, dev_log);
  FTAR_CHECK_HIP(hipGetLastError());
  return FTAR_SUCCESS;
}

namespace {
__global__ void noop_kernel() {}
}  // namespace

ftar_status_t launch_noop(hipStream_t stream) {
  FTAR_LAUNCH(noop_kernel, dim3(1), dim3(64), 0, stream);
  FTAR_CHECK_HIP(hipGetLastError());
  return FTAR_SUCCESS;
}

namespace {
// the LDS-staged kernel up to k = HOT, or (lds == false: the peer forms' ":vec" A/B) only at k = 2
template <class Tr, int HOT>
hipError_t tr(bool lds, const void* const* srcs, int k, void* dst, size_t count, hipStream_t s) {
  return lds ? launch_tr<Tr, HOT>(srcs, k, dst, count, s) : launch_tr<Tr, 0>(srcs, k, dst, count, s);
}
}  // namespace

// The LDS-staged kernel with K = 1 on one-wave workgroups of one tile (U = 1, W = 1; byte traits, so any
// dtype): 6,530 vs 6,012 GB/s for the multi-segment copy kernel on cold 256 MiB buffers, the best of 17
// (U, W) shapes (tools/kbench_cold.py --ks 1, profiles/r03/kbench_copy.log).  Sources and destinations
// whose 16-byte alignments differ take the copy kernel, which handles any alignment.
ftar_status_t launch_copy(const void* src, void* dst, size_t bytes, hipStream_t s) {
  if (!bytes || src == dst) return FTAR_SUCCESS;
  const uintptr_t mis = reinterpret_cast<uintptr_t>(dst) & 15;
  if ((reinterpret_cast<uintptr_t>(src) & 15) != mis) {
    const Segment seg{src, dst, bytes};
    return launch_gather(&seg, 1, s);
  }
  size_t head = mis ? 16 - mis : 0;
  if (head > bytes) head = bytes;
  const size_t nvec = (bytes - head) / 16;
  const int tail = (int)(bytes - head - nvec * 16);
  const void* srcs[1] = {src};
  FTAR_CHECK_HIP((launch_lds<U8Sum, 1, 1, 1>(srcs, dst, nvec, s, (int)head, tail)));
  return FTAR_SUCCESS;
}

ftar_status_t launch_reduce(const void* const* srcs, int k, void* dst, size_t count, ftar_dtype_t dt, ftar_op_t op,
                            hipStream_t s, bool round_each, const int* shape, int nlevels, bool lds) {
  if (k < 1 || k > FTAR_MAX_K || !srcs || !dst) return FTAR_ERR_INVALID_ARG;
  if (!dtype_op_supported(dt, op)) return FTAR_ERR_UNSUPPORTED;
  if (count == 0) return FTAR_SUCCESS;
  for (int j = 0; j < k; ++j)
    if (!srcs[j]) return FTAR_ERR_INVALID_ARG;
  if (k == 1)  // vector_add/reduce_sum.h:36-47: a copy (a streaming kernel, not the DMA blit)
    return launch_copy(srcs[0], dst, count * dtype_size(dt), s);
  hipError_t e = hipErrorInvalidValue;
  if (nlevels > 1 && op == FTAR_SUM && (dt == FTAR_FLOAT32 || dt == FTAR_FLOAT64 || dt == FTAR_BFLOAT16)) {
    TreeCode tc;
    if (!shape || !make_tree_code(shape, nlevels, k, &tc)) return FTAR_ERR_INVALID_ARG;
    switch (dt) {
      case FTAR_FLOAT32: e = launch_tree<F32Sum>(srcs, k, tc, shape, nlevels, dst, count, s, lds); break;
      case FTAR_FLOAT64: e = launch_tree<F64Sum>(srcs, k, tc, shape, nlevels, dst, count, s, false); break;
      default: e = launch_tree<BF16Sum>(srcs, k, tc, shape, nlevels, dst, count, s, lds); break;
    }
    FTAR_CHECK_HIP(e);
    return FTAR_SUCCESS;
  }
  if (op == FTAR_SUM) {
    switch (dt) {
      case FTAR_FLOAT32: e = tr<F32Sum, 16>(lds, srcs, k, dst, count, s); break;
      case FTAR_BFLOAT16:
        e = round_each && k > 2 ? tr<BF16SumHop, 16>(lds, srcs, k, dst, count, s)
                                : tr<BF16Sum, 16>(lds, srcs, k, dst, count, s);
        break;
      case FTAR_FLOAT64: e = tr<F64Sum, 8>(lds, srcs, k, dst, count, s); break;
      case FTAR_UINT8: case FTAR_INT8: e = tr<U8Sum, 8>(lds, srcs, k, dst, count, s); break;
      case FTAR_UINT16: case FTAR_INT16: e = tr<U16Sum, 8>(lds, srcs, k, dst, count, s); break;
      case FTAR_INT32: e = tr<U32Sum, 8>(lds, srcs, k, dst, count, s); break;
      case FTAR_INT64: e = tr<U64Sum, 8>(lds, srcs, k, dst, count, s); break;
      case FTAR_BOOL: e = tr<BoolSum, 8>(lds, srcs, k, dst, count, s); break;
    }
  } else {
    switch (dt) {
      case FTAR_UINT8: case FTAR_INT8: e = tr<Band<unsigned char>, 8>(lds, srcs, k, dst, count, s); break;
      case FTAR_UINT16: case FTAR_INT16: e = tr<Band<unsigned short>, 8>(lds, srcs, k, dst, count, s); break;
      case FTAR_INT32: e = tr<Band<unsigned>, 8>(lds, srcs, k, dst, count, s); break;
      case FTAR_INT64: e = tr<Band<unsigned long long>, 8>(lds, srcs, k, dst, count, s); break;
      default: return FTAR_ERR_UNSUPPORTED;
    }
  }
  FTAR_CHECK_HIP(e);
  return FTAR_SUCCESS;
}

}  // namespace ftar

// The kernel the reduce/copy launchers last launched on the calling thread, demangled the way rocprofv3
// prints kernel names ("void ftar::(anonymous namespace)::reduce_lds_kernel<...>(...)"); bench.py
// ties the PMC traffic it reports to this symbol.  Returns the length needed (excluding the NUL), or
// -1 when nothing was launched on this thread.
extern "C" long ftar_debug_last_kernel(char* buf, size_t buflen) {
  const void* k = ftar::g_last_kernel;
  if (!k) return -1;
  const char* raw = hipKernelNameRefByPtr(k, nullptr);
  if (!raw) return -1;
  int status = 0;
  char* dem = abi::__cxa_demangle(raw, nullptr, nullptr, &status);
  const char* name = status == 0 && dem ? dem : raw;
  const size_t need = strlen(name);
  if (buf && buflen) {
    const size_t m = need < buflen - 1 ? need : buflen - 1;
    memcpy(buf, name, m);
    buf[m] = 0;
  }
  free(dem);
  return (long)need;
}
