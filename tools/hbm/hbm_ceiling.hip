// HBM ceilings on this MI355X (tool, not product): what streaming read-only,
// write-only, copy (1R:1W) and 2R:1W (the k = 2 reduce's mix) kernels reach,
// same launch shape as reduce_vec_kernel (256 threads, 2 x 16 B per lane per
// stream, nontemporal loads, one-shot grid).  Prints one JSON line per test.
//   hipcc --offload-arch=gfx950 -O3 -o hbm_ceiling hbm_ceiling.hip
//   ./hbm_ceiling [elements] [reps] [rounds] [sets]
// sets > 1 rotates the launches over that many disjoint buffer sets, so a
// launch never finds its data in the 256 MB Infinity Cache (MALL) from the
// previous one.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kT = 256, kU = 2;

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                  \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

__global__ void __launch_bounds__(kT) read2(const u32x4* a, const u32x4* b, u32x4* sink, size_t nvec) {
  size_t v = (size_t)blockIdx.x * (kU * kT) + threadIdx.x;
  u32x4 acc = {0, 0, 0, 0};
  for (int u = 0; u < kU; ++u, v += kT)
    if (v < nvec) acc ^= __builtin_nontemporal_load(a + v) ^ __builtin_nontemporal_load(b + v);
  if ((acc.x & 0xffffff) == 0x123457 && acc.y == 7) sink[blockIdx.x] = acc;  // never true for the data below
}
__global__ void __launch_bounds__(kT) write1(u32x4* d, size_t nvec) {
  size_t v = (size_t)blockIdx.x * (kU * kT) + threadIdx.x;
  for (int u = 0; u < kU; ++u, v += kT)
    if (v < nvec) d[v] = u32x4{(unsigned)v, 1u, 2u, 3u};
}
__global__ void __launch_bounds__(kT) copy1(const u32x4* a, u32x4* d, size_t nvec) {
  size_t v = (size_t)blockIdx.x * (kU * kT) + threadIdx.x;
  u32x4 x[kU];
  for (int u = 0; u < kU; ++u) x[u] = v + u * kT < nvec ? __builtin_nontemporal_load(a + v + u * kT) : u32x4{0, 0, 0, 0};
  for (int u = 0; u < kU; ++u)
    if (v + u * kT < nvec) d[v + u * kT] = x[u];
}
__global__ void __launch_bounds__(kT) add2(const u32x4* a, const u32x4* b, u32x4* d, size_t nvec) {
  size_t v = (size_t)blockIdx.x * (kU * kT) + threadIdx.x;
  u32x4 x[kU], y[kU];
  for (int u = 0; u < kU; ++u) {
    x[u] = v + u * kT < nvec ? __builtin_nontemporal_load(a + v + u * kT) : u32x4{0, 0, 0, 0};
    y[u] = v + u * kT < nvec ? __builtin_nontemporal_load(b + v + u * kT) : u32x4{0, 0, 0, 0};
  }
  for (int u = 0; u < kU; ++u)
    if (v + u * kT < nvec) d[v + u * kT] = x[u] + y[u];
}

template <int U>
__global__ void __launch_bounds__(kT) copy_nt(const u32x4* a, u32x4* d, size_t nvec) {
  size_t v = (size_t)blockIdx.x * (U * kT) + threadIdx.x;
  u32x4 x[U];
  for (int u = 0; u < U; ++u) x[u] = v + u * kT < nvec ? __builtin_nontemporal_load(a + v + u * kT) : u32x4{0, 0, 0, 0};
  for (int u = 0; u < U; ++u)
    if (v + u * kT < nvec) __builtin_nontemporal_store(x[u], d + v + u * kT);
}
__global__ void __launch_bounds__(kT) write_nt(u32x4* d, size_t nvec) {
  size_t v = (size_t)blockIdx.x * (kU * kT) + threadIdx.x;
  for (int u = 0; u < kU; ++u, v += kT)
    if (v < nvec) __builtin_nontemporal_store(u32x4{(unsigned)v, 1u, 2u, 3u}, d + v);
}

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 0) : (size_t)1 << 26;  // fp32 elements per stream
  const int reps = argc > 2 ? atoi(argv[2]) : 20, rounds = argc > 3 ? atoi(argv[3]) : 5;
  const int sets = argc > 4 ? atoi(argv[4]) : 1;
  const size_t nvec = n / 4, bytes = n * 4;
  u32x4 *A[16], *B[16], *D[16], *sink;
  for (int i = 0; i < sets && i < 16; ++i) {
    CHECK(hipMalloc(&A[i], bytes));
    CHECK(hipMalloc(&B[i], bytes));
    CHECK(hipMalloc(&D[i], bytes));
    CHECK(hipMemset(A[i], 1, bytes));
    CHECK(hipMemset(B[i], 2, bytes));
  }
  const unsigned blocks = (unsigned)((nvec + kU * kT - 1) / (kU * kT));
  CHECK(hipMalloc(&sink, (size_t)blocks * sizeof(u32x4)));
  int cur = 0;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const char* names[8] = {"read 2 streams", "write 1 stream", "copy 1R:1W", "add 2R:1W (k=2 reduce mix)",
                          "write 1 stream, nt stores", "copy 1R:1W, nt stores, 2/lane", "copy 1R:1W, nt stores, 4/lane",
                          "hipMemcpyAsync D2D"};
  const double traffic[8] = {2.0 * bytes, 1.0 * bytes, 2.0 * bytes, 3.0 * bytes, 1.0 * bytes, 2.0 * bytes, 2.0 * bytes,
                             2.0 * bytes};
  for (int r = 0; r < rounds; ++r)
    for (int t = 0; t < 8; ++t) {
      auto launch = [&] {
        const int i = cur++ % sets;
        u32x4 *a = A[i], *b = B[i], *d = D[i];
        if (t == 0) hipLaunchKernelGGL(read2, dim3(blocks), dim3(kT), 0, 0, a, b, sink, nvec);
        if (t == 1) hipLaunchKernelGGL(write1, dim3(blocks), dim3(kT), 0, 0, d, nvec);
        if (t == 2) hipLaunchKernelGGL(copy1, dim3(blocks), dim3(kT), 0, 0, a, d, nvec);
        if (t == 3) hipLaunchKernelGGL(add2, dim3(blocks), dim3(kT), 0, 0, a, b, d, nvec);
        if (t == 4) hipLaunchKernelGGL(write_nt, dim3(blocks), dim3(kT), 0, 0, d, nvec);
        if (t == 5) hipLaunchKernelGGL(copy_nt<2>, dim3(blocks), dim3(kT), 0, 0, a, d, nvec);
        if (t == 6) hipLaunchKernelGGL(copy_nt<4>, dim3((blocks + 1) / 2), dim3(kT), 0, 0, a, d, nvec);
        if (t == 7) (void)hipMemcpyAsync(d, a, bytes, hipMemcpyDeviceToDevice, 0);
      };
      for (int i = 0; i < 3; ++i) launch();
      CHECK(hipEventRecord(e0, 0));
      for (int i = 0; i < reps; ++i) launch();
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double per = ms / reps;
      printf("{\"round\": %d, \"test\": \"%s\", \"elements\": %zu, \"sets\": %d, \"us\": %.2f, \"GBps\": %.1f}\n", r,
             names[t], n, sets, per * 1e3, traffic[t] / (per * 1e-3) / 1e9);
    }
  return 0;
}
