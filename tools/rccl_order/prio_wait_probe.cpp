// prio_wait_probe — does a stream wait on an event recorded after an H2D copy on a HIGH-PRIORITY stream
// hold the waiting stream until the copy has landed?  (the host path's copy streams.)
//
// Each iteration copies a pinned host buffer holding pattern i % 2 into one device buffer on the copy stream
// (high priority, or plain for the control), records an event there, makes a plain stream wait on it and
// launches a kernel on the plain stream that counts the words of the device buffer that do not hold
// pattern i % 2.  A wait that let the kernel start before the copy landed shows as a nonzero count.
//
// --reverse: the other direction -- a kernel on a plain stream writes pattern i % 2 into the device buffer
// (after spinning ~1 ms, so its writes land late), records an event; the copy stream (high priority, or
// plain) waits on it and copies the buffer D2H into pinned memory; the host counts the words that do not
// hold pattern i % 2 (a copy that started before the kernel ended).  The host path's D2H waits this way on
// its gather kernel.
//
// Usage: prio_wait_probe [--plain] [--reverse] [--iters N] [--mib M]     (prints one JSON line)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CHECK(x)                                                                                \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));          \
      exit(2);                                                                                  \
    }                                                                                           \
  } while (0)

// every block spins ~spin_ticks of the wall clock, then writes its share of buf
__global__ void late_fill_kernel(unsigned* buf, size_t n, unsigned v, unsigned long long spin_ticks) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < spin_ticks) __builtin_amdgcn_s_sleep(8);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) buf[i] = v;
}

// every word of buf against `want`; mismatches of iteration `it` into bad[it] (a vector atomic per wave
// that found any)
__global__ void count_kernel(const unsigned* buf, size_t n, unsigned want, unsigned long long* bad, int it) {
  unsigned long long mine = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    mine += buf[i] != want;
  for (int off = 32; off > 0; off >>= 1) mine += __shfl_down(mine, off);
  if ((threadIdx.x & 63) == 0 && mine) atomicAdd(&bad[it], mine);
}

int main(int argc, char** argv) {
  bool plain = false, reverse = false;
  int iters = 200;
  size_t mib = 256;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "--plain") plain = true;
    else if (a == "--reverse") reverse = true;
    else if (a == "--iters" && i + 1 < argc) iters = atoi(argv[++i]);
    else if (a == "--mib" && i + 1 < argc) mib = (size_t)atol(argv[++i]);
  }
  const size_t bytes = mib << 20, n = bytes / 4;
  CHECK(hipSetDevice(0));
  unsigned* host[2];
  for (int p = 0; p < 2; ++p) {
    CHECK(hipHostMalloc((void**)&host[p], bytes, hipHostMallocDefault));
    const unsigned v = p ? 0x22222222u : 0x11111111u;
    for (size_t i = 0; i < n; ++i) host[p][i] = v;
  }
  unsigned* dev = nullptr;
  unsigned long long* bad = nullptr;
  CHECK(hipMalloc(&dev, bytes));
  CHECK(hipMalloc(&bad, sizeof(unsigned long long) * iters));
  CHECK(hipMemset(bad, 0, sizeof(unsigned long long) * iters));
  int lo = 0, hi = 0;
  CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  hipStream_t copy_s, work_s;
  if (plain) CHECK(hipStreamCreateWithFlags(&copy_s, hipStreamNonBlocking));
  else CHECK(hipStreamCreateWithPriority(&copy_s, hipStreamNonBlocking, hi));
  CHECK(hipStreamCreateWithFlags(&work_s, hipStreamNonBlocking));
  hipEvent_t copied, checked;
  CHECK(hipEventCreateWithFlags(&copied, hipEventDisableTiming));
  CHECK(hipEventCreateWithFlags(&checked, hipEventDisableTiming));
  CHECK(hipDeviceSynchronize());
  if (reverse) {
    int khz = 0;
    CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
    int failed = 0;
    unsigned long long words = 0;
    for (int it = 0; it < iters; ++it) {
      const unsigned v = it % 2 ? 0x22222222u : 0x11111111u;
      hipLaunchKernelGGL(late_fill_kernel, dim3(1024), dim3(256), 0, work_s, dev, n, v, (unsigned long long)khz);  // ~1 ms
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(copied, work_s));
      CHECK(hipStreamWaitEvent(copy_s, copied, 0));
      CHECK(hipMemcpyAsync(host[0], dev, bytes, hipMemcpyDeviceToHost, copy_s));
      CHECK(hipStreamSynchronize(copy_s));
      unsigned long long bad_words = 0;
      for (size_t i = 0; i < n; ++i) bad_words += host[0][i] != v;
      failed += bad_words != 0;
      words += bad_words;
      CHECK(hipStreamSynchronize(work_s));
    }
    printf("{\"direction\": \"kernel then D2H\", \"copy_stream\": \"%s\", \"iters\": %d, \"mib\": %zu, "
           "\"iterations_with_stale_words\": %d, \"stale_words\": %llu}\n",
           plain ? "plain" : "high-priority", iters, mib, failed, words);
    return 0;
  }
  for (int it = 0; it < iters; ++it) {
    CHECK(hipStreamWaitEvent(copy_s, checked, 0));  // the previous check has read the buffer
    CHECK(hipMemcpyAsync(dev, host[it % 2], bytes, hipMemcpyHostToDevice, copy_s));
    CHECK(hipEventRecord(copied, copy_s));
    CHECK(hipStreamWaitEvent(work_s, copied, 0));
    hipLaunchKernelGGL(count_kernel, dim3(1024), dim3(256), 0, work_s, dev, n, it % 2 ? 0x22222222u : 0x11111111u,
                       bad, it);
    CHECK(hipGetLastError());
    CHECK(hipEventRecord(checked, work_s));
  }
  CHECK(hipDeviceSynchronize());
  std::vector<unsigned long long> h(iters);
  CHECK(hipMemcpy(h.data(), bad, sizeof(unsigned long long) * iters, hipMemcpyDeviceToHost));
  int failed = 0;
  unsigned long long words = 0;
  for (int it = 0; it < iters; ++it) {
    failed += h[it] != 0;
    words += h[it];
  }
  printf("{\"copy_stream\": \"%s\", \"iters\": %d, \"mib\": %zu, \"iterations_with_stale_words\": %d, "
         "\"stale_words\": %llu}\n", plain ? "plain" : "high-priority", iters, mib, failed, words);
  return 0;
}
