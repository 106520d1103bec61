// queue_probe — which of a process's HIP streams share a hardware queue?  
//
// HIP gives a process at most GPU_MAX_HW_QUEUES hardware (AQL) queues (4 by default); further streams share
// them.  Kernels on one queue run in issue order, so a kernel that waits for a peer (an RCCL p2p kernel)
// holds up everything queued behind it on that queue, whichever stream issued it.  This probe brings up K
// ftar communicators (1-rank RCCL ones, so RCCL's own streams exist as in the product), collects their
// internal streams (comm, reduce, H2D, D2H) plus a caller stream, and for every ordered pair (X, Y) launches
// a kernel on X that spins until released (or 2 s pass), then a trivial kernel on Y: if Y's kernel cannot
// finish within 300 ms while X spins, X and Y share a queue.  Optional extra streams: a CU-masked stream
// with every CU ("masked"), which the runtime gives a queue of its own, and a high-priority stream ("prio");
// the legacy NULL stream ("null", the caller stream of the engine stress driver): a blocking stream such as
// the masked one also waits for it (and it for them) without sharing a queue, which the pairs show as well.
//
// Usage: queue_probe [--comms K] [--masked] [--prio [N]] [--extra N] [--null] [--host-call] [--ipc]
//   --host-call: one host-buffer call on each communicator first, so its H2D / D2H streams exist;
//   --ipc: host-bootstrapped 1-rank communicators (the MPI drop-in's ipc transport) instead of RCCL ones.
//   --prio N: N high-priority streams; --extra N: N plain streams created after the communicators (as the
//   host path's H2D / D2H streams are, at the first host-buffer call).  Prints "SHARE <x> <y> yes|no" and a summary.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "ftar.h"

extern "C" ftar_status_t ftar_debug_comm_streams(ftar_comm_t comm, void** streams4);

#define CHECK(x)                                                                                \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));          \
      exit(2);                                                                                  \
    }                                                                                           \
  } while (0)

// every wave reaches the exit: the host flag, or the wall-clock limit
// (a system-scope atomic load, so the host's release is seen)
__global__ void spin_kernel(int* flag, unsigned long long limit_ticks) {
  const unsigned long long t0 = wall_clock64();
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0 &&
         wall_clock64() - t0 < limit_ticks)
    __builtin_amdgcn_s_sleep(8);
}

// one vector store per lane
__global__ void marker_kernel(int* out) { out[threadIdx.x] = 1; }

int main(int argc, char** argv) {
  int ncomms = 1;
  bool masked = false, null_stream = false;
  int prio = 0, extra = 0;
  bool host_call = false, ipc = false;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "--comms" && i + 1 < argc) ncomms = atoi(argv[++i]);
    else if (a == "--masked") masked = true;
    else if (a == "--prio") prio = (i + 1 < argc && argv[i + 1][0] != '-') ? atoi(argv[++i]) : 1;
    else if (a == "--extra" && i + 1 < argc) extra = atoi(argv[++i]);
    else if (a == "--host-call") host_call = true;
    else if (a == "--ipc") ipc = true;
    else if (a == "--null") null_stream = true;
  }
  CHECK(hipSetDevice(0));
  int khz = 0;
  CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  const unsigned long long limit = (unsigned long long)khz * 2000ull;  // 2 s

  std::vector<std::pair<std::string, hipStream_t>> st;
  hipStream_t user;
  CHECK(hipStreamCreateWithFlags(&user, hipStreamNonBlocking));
  st.emplace_back("caller", user);
  if (null_stream) st.emplace_back("null", static_cast<hipStream_t>(nullptr));
  std::vector<ftar_comm_t> comms;
  for (int c = 0; c < ncomms; ++c) {
    ftar_unique_id_t id;
    ftar_comm_t comm = nullptr;
    auto one_rank_allgather = [](const void* mine, void* all, size_t bytes, void*) -> int {
      memcpy(all, mine, bytes);
      return 0;
    };
    const ftar_status_t made = ipc ? ftar_comm_init_host(&comm, 1, 0, 0, one_rank_allgather, nullptr)
                                   : ftar_get_unique_id(&id) == FTAR_SUCCESS ? ftar_comm_init_rank(&comm, 1, id, 0, 0)
                                                                             : FTAR_ERR_INTERNAL;
    if (made != FTAR_SUCCESS) {
      fprintf(stderr, "communicator %d: %s\n", c, ftar_last_error());
      return 2;
    }
    comms.push_back(comm);
    if (host_call) {  // creates the communicator's H2D / D2H streams
      float hx = 1.f;
      if (ftar_allreduce_host(nullptr, &hx, 1, FTAR_FLOAT32, FTAR_SUM, nullptr, comm, user) != FTAR_SUCCESS) {
        fprintf(stderr, "host call %d: %s\n", c, ftar_last_error());
        return 2;
      }
      CHECK(hipStreamSynchronize(user));
    }
    void* s4[4] = {};
    ftar_debug_comm_streams(comm, s4);
    const char* names[4] = {"comm", "reduce", "h2d", "d2h"};
    for (int j = 0; j < 4; ++j)
      if (s4[j]) st.emplace_back("c" + std::to_string(c) + "." + names[j], static_cast<hipStream_t>(s4[j]));
  }
  if (masked) {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0u);
    for (int i = 0; i < cus; ++i) mask[(size_t)i / 32] |= 1u << (i % 32);
    hipStream_t m;
    CHECK(hipExtStreamCreateWithCUMask(&m, (uint32_t)mask.size(), mask.data()));
    st.emplace_back("masked_all", m);
  }
  for (int e = 0; e < extra; ++e) {
    hipStream_t x;
    CHECK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    st.emplace_back("extra" + std::to_string(e), x);
  }
  for (int e = 0; e < prio; ++e) {
    int lo = 0, hi = 0;
    CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    hipStream_t p;
    CHECK(hipStreamCreateWithPriority(&p, hipStreamNonBlocking, hi));
    st.emplace_back(prio == 1 ? std::string("prio_high") : "prio_high" + std::to_string(e), p);
  }

  int* flag = nullptr;
  int* out = nullptr;
  CHECK(hipHostMalloc((void**)&flag, sizeof(int), hipHostMallocCoherent | hipHostMallocMapped));
  CHECK(hipMalloc(&out, 64 * sizeof(int)));
  const char* q = getenv("GPU_MAX_HW_QUEUES");
  printf("queue_probe: %zu streams, %d communicators, GPU_MAX_HW_QUEUES=%s\n", st.size(), ncomms, q ? q : "(default)");
  int shared_pairs = 0;
  for (size_t x = 0; x < st.size(); ++x)
    for (size_t y = 0; y < st.size(); ++y) {
      if (x == y) continue;
      __atomic_store_n(flag, 0, __ATOMIC_SEQ_CST);
      hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, st[x].second, flag, limit);
      CHECK(hipGetLastError());
      hipLaunchKernelGGL(marker_kernel, dim3(1), dim3(64), 0, st[y].second, out);
      CHECK(hipGetLastError());
      const auto t0 = std::chrono::steady_clock::now();
      bool done = false;
      while (!done && std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(300)) {
        done = hipStreamQuery(st[y].second) == hipSuccess;
        if (!done) std::this_thread::sleep_for(std::chrono::milliseconds(1));
      }
      __atomic_store_n(flag, 1, __ATOMIC_SEQ_CST);
      CHECK(hipStreamSynchronize(st[x].second));
      CHECK(hipStreamSynchronize(st[y].second));
      printf("SHARE %s %s %s\n", st[x].first.c_str(), st[y].first.c_str(), done ? "no" : "yes");
      shared_pairs += !done;
    }
  printf("queue_probe: %d of %zu ordered pairs blocked\n", shared_pairs, st.size() * (st.size() - 1));
  fflush(stdout);
  for (ftar_comm_t c : comms) ftar_comm_destroy(c);
  (void)hipHostFree(flag);
  (void)hipFree(out);
  return 0;
}
