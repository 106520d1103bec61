// ftar_capture_check — the in-process group AllReduce (ftar_allreduce_group on a
// ftar_comm_init_local group) captured into one HIP graph from plain C++,
// without torch: decides whether a crash in hipStreamEndCapture belongs to the
// HIP runtime torch bundles (7.0) or to ftar.  Replays on fresh inputs and
// compares every rank's output with an uncaptured call on the same inputs.
//   ftar_capture_check P TOPO N CHUNK [shared [LONELY]]  (TOPO "1" = ring, else stage widths;
//   shared: every rank's call on the capture stream itself, no per-rank fork)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ftar.h"

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));        \
      exit(2);                                                                                  \
    }                                                                                           \
  } while (0)
#define FT(x)                                                                                   \
  do {                                                                                          \
    ftar_status_t s_ = (x);                                                                     \
    if (s_ != FTAR_SUCCESS) {                                                                   \
      fprintf(stderr, "%s:%d %s: %s (%s)\n", __FILE__, __LINE__, #x, ftar_status_string(s_),   \
              ftar_last_error());                                                               \
      exit(3);                                                                                  \
    }                                                                                           \
  } while (0)

int main(int argc, char** argv) {
  const int P = argc > 1 ? atoi(argv[1]) : 2;
  const char* ts = argc > 2 ? argv[2] : "1";
  const size_t n = argc > 3 ? strtoull(argv[3], nullptr, 0) : 10007;
  const size_t chunk = argc > 4 ? strtoull(argv[4], nullptr, 0) : 0;
  const bool shared = argc > 5 && !strcmp(argv[5], "shared");
  int dv = 0;
  CK(hipRuntimeGetVersion(&dv));
  fprintf(stderr, "HIP runtime %d\n", dv);
  std::vector<ftar_comm_t> comms(P);
  FT(ftar_comm_init_local(comms.data(), P, nullptr));
  ftar_topo_t topo;
  FT(ftar_topo_parse(ts, argc > 6 ? argv[6] : "0", P, &topo));
  for (auto c : comms) {
    if (chunk) FT(ftar_comm_set_chunk_bytes(c, chunk));
  }
  std::vector<float*> x(P), y(P), ref(P);
  std::vector<void*> xv(P), yv(P), rv(P);
  std::vector<std::vector<float>> hx(P, std::vector<float>(n));
  for (int r = 0; r < P; ++r) {
    CK(hipMalloc(&x[r], n * 4));
    CK(hipMalloc(&y[r], n * 4));
    CK(hipMalloc(&ref[r], n * 4));
    xv[r] = x[r];
    yv[r] = y[r];
    rv[r] = ref[r];
  }
  auto fill = [&](int round) {
    for (int r = 0; r < P; ++r) {
      for (size_t i = 0; i < n; ++i) hx[r][i] = (float)((i * 2654435761u + r * 40503u + round * 977u) % 1000) / 7.0f;
      CK(hipMemcpy(x[r], hx[r].data(), n * 4, hipMemcpyHostToDevice));
    }
  };
  std::vector<const void*> xc(xv.begin(), xv.end());
  fill(0);
  FT(ftar_allreduce_group(xc.data(), yv.data(), n, FTAR_FLOAT32, FTAR_SUM, &topo, comms.data(), P, nullptr));
  CK(hipDeviceSynchronize());
  fprintf(stderr, "warm-up done\n");

  hipStream_t s0;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  std::vector<hipStream_t> rs(P);
  std::vector<void*> rsv(P);
  std::vector<hipEvent_t> join(P);
  hipEvent_t fork;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  for (int r = 0; r < P; ++r) {
    CK(hipStreamCreateWithFlags(&rs[r], hipStreamNonBlocking));
    CK(hipEventCreateWithFlags(&join[r], hipEventDisableTiming));
    rsv[r] = shared ? (void*)s0 : (void*)rs[r];
  }
  CK(hipStreamBeginCapture(s0, hipStreamCaptureModeRelaxed));
  CK(hipEventRecord(fork, s0));
  if (!shared)
    for (auto s : rs) CK(hipStreamWaitEvent(s, fork, 0));
  FT(ftar_allreduce_group(xc.data(), yv.data(), n, FTAR_FLOAT32, FTAR_SUM, &topo, comms.data(), P, rsv.data()));
  fprintf(stderr, "group call issued\n");
  for (int r = 0; r < P && !shared; ++r) {
    CK(hipEventRecord(join[r], rs[r]));
    CK(hipStreamWaitEvent(s0, join[r], 0));
  }
  hipGraph_t graph;
  CK(hipStreamEndCapture(s0, &graph));
  size_t nodes = 0;
  CK(hipGraphGetNodes(graph, nullptr, &nodes));
  fprintf(stderr, "capture ended: %zu nodes\n", nodes);
  hipGraphExec_t exe;
  CK(hipGraphInstantiate(&exe, graph, nullptr, nullptr, 0));
  std::vector<float> a(n), b(n);
  for (int round = 1; round <= 3; ++round) {
    fill(round);
    FT(ftar_allreduce_group(xc.data(), rv.data(), n, FTAR_FLOAT32, FTAR_SUM, &topo, comms.data(), P, nullptr));
    CK(hipMemset(y[0], 0xff, n * 4));
    CK(hipDeviceSynchronize());
    CK(hipGraphLaunch(exe, s0));
    CK(hipStreamSynchronize(s0));
    for (int r = 0; r < P; ++r) {
      CK(hipMemcpy(a.data(), y[r], n * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(b.data(), ref[r], n * 4, hipMemcpyDeviceToHost));
      if (memcmp(a.data(), b.data(), n * 4) != 0) {
        printf("replay %d rank %d differs from the uncaptured call\n", round, r);
        return 1;
      }
    }
  }
  for (auto c : comms) ftar_comm_destroy(c);
  printf("group capture ok: P=%d topo=%s n=%zu chunk=%zu, %zu nodes, 3 replays bit-identical\n", P, ts, n, chunk,
         nodes);
  return 0;
}
