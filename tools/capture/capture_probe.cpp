// capture_probe — which multi-stream / multi-thread stream-capture patterns the
// HIP runtime accepts (diagnostic for the in-process group capture).
// Each case runs in its own process (argv[1] = case), captures into one graph
// from stream s0 (relaxed mode), instantiates, replays twice and checks the
// data.  Prints "case N ok" or dies.
//   1  one thread: fork s1 from s0, kernel + D2D memcpy on s1, join
//   2  one thread: s1 -> event -> s2 waits, memcpy on s2, both joined
//   3  as 2, the s2 part issued from a second thread (turns via a mutex)
//   4  one thread: one event recorded twice in the capture (two waits)
//   5  as 3 but s2 first joins the capture by waiting on an event recorded on
//      a stream forked in ANOTHER thread, then s2's own event joins s0
//   6  one thread: a stream joins via an event wait and is joined back
//      only through a second stream (chain s0 -> s1 -> s2 -> s0)
//   7  one thread: a wait inside the capture on an event last recorded
//      OUTSIDE it (before hipStreamBeginCapture)
//   8  one thread: an event waited on, then RE-RECORDED later in the capture
//      at a point that depends on the waiter's later work (s1 record e1;
//      s2 wait e1, memcpy, record e2; s1 wait e2, kernel, record e1 again)
//   9  as 3, the other thread calls hipSetDevice first and launches a kernel
//      on s2 after the memcpy (b = a + 1)
//  10  as 9, and the other thread also calls hipStreamIsCapturing(s2) and
//      creates a fresh event in the capture for its join
//  11  one event re-recorded on ANOTHER stream: s1 record e1; s2 wait e1,
//      memcpy; s2 record e1 (same event); s1 wait e1; kernel on s1
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <thread>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                     \
    }                                                                              \
  } while (0)

__global__ void add_one(float* p, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) p[i] += 1.0f;
}

int main(int argc, char** argv) {
  const int cs = argc > 1 ? atoi(argv[1]) : 1;
  const size_t n = 1 << 20;
  float *a, *b, *c;
  CK(hipMalloc(&a, n * 4));
  CK(hipMalloc(&b, n * 4));
  CK(hipMalloc(&c, n * 4));
  hipStream_t s0, s1, s2;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t fork, e1, e2, join1, join2;
  for (hipEvent_t* e : {&fork, &e1, &e2, &join1, &join2}) CK(hipEventCreateWithFlags(e, hipEventDisableTiming));
  std::mutex turn;

  if (cs == 7) {
    CK(hipEventRecord(e2, s2));  // recorded before the capture begins
    CK(hipStreamSynchronize(s2));
  }
  CK(hipStreamBeginCapture(s0, hipStreamCaptureModeRelaxed));
  CK(hipEventRecord(fork, s0));
  CK(hipStreamWaitEvent(s1, fork, 0));
  add_one<<<n / 256, 256, 0, s1>>>(a, n);  // a += 1
  auto part2 = [&]() {  // s2: after s1's kernel, b = a; joined
    std::lock_guard<std::mutex> g(turn);
    CK(hipStreamWaitEvent(s2, e1, 0));
    CK(hipMemcpyAsync(b, a, n * 4, hipMemcpyDeviceToDevice, s2));
    CK(hipEventRecord(join2, s2));
  };
  switch (cs) {
    case 1:
      CK(hipMemcpyAsync(b, a, n * 4, hipMemcpyDeviceToDevice, s1));
      break;
    case 7:
      CK(hipStreamWaitEvent(s1, e2, 0));
      CK(hipMemcpyAsync(b, a, n * 4, hipMemcpyDeviceToDevice, s1));
      break;
    case 2:
    case 3:
    case 5: {
      CK(hipEventRecord(e1, s1));
      if (cs == 2) {
        part2();
      } else {
        std::thread t(part2);
        t.join();
      }
      CK(hipStreamWaitEvent(s0, join2, 0));
      break;
    }
    case 4:
      CK(hipEventRecord(e1, s1));
      CK(hipStreamWaitEvent(s2, e1, 0));
      add_one<<<n / 256, 256, 0, s1>>>(a, n);  // a += 1 again
      CK(hipEventRecord(e1, s1));             // re-recorded
      CK(hipStreamWaitEvent(s2, e1, 0));
      CK(hipMemcpyAsync(b, a, n * 4, hipMemcpyDeviceToDevice, s2));
      CK(hipEventRecord(join2, s2));
      CK(hipStreamWaitEvent(s0, join2, 0));
      break;
    case 8:
      CK(hipEventRecord(e1, s1));
      CK(hipStreamWaitEvent(s2, e1, 0));
      CK(hipMemcpyAsync(b, a, n * 4, hipMemcpyDeviceToDevice, s2));
      CK(hipEventRecord(e2, s2));
      CK(hipStreamWaitEvent(s1, e2, 0));
      add_one<<<n / 256, 256, 0, s1>>>(c, n);
      CK(hipEventRecord(e1, s1));  // e1 again, after work that depends on the earlier waiter
      CK(hipEventRecord(join2, s2));
      CK(hipStreamWaitEvent(s0, join2, 0));
      break;
    case 9:
    case 10: {
      CK(hipEventRecord(e1, s1));
      hipEvent_t fresh = nullptr;
      std::thread t([&]() {
        std::lock_guard<std::mutex> g(turn);
        CK(hipSetDevice(0));
        CK(hipStreamWaitEvent(s2, e1, 0));
        CK(hipMemcpyAsync(b, a, n * 4, hipMemcpyDeviceToDevice, s2));
        add_one<<<n / 256, 256, 0, s2>>>(b, n);
        CK(hipGetLastError());
        if (cs == 10) {
          hipStreamCaptureStatus st;
          CK(hipStreamIsCapturing(s2, &st));
          if (st != hipStreamCaptureStatusActive) fprintf(stderr, "s2 not capturing?\n");
          CK(hipEventCreateWithFlags(&fresh, hipEventDisableTiming));
          CK(hipEventRecord(fresh, s2));
        } else {
          CK(hipEventRecord(join2, s2));
        }
      });
      t.join();
      CK(hipStreamWaitEvent(s0, cs == 10 ? fresh : join2, 0));
      break;
    }
    case 11:
      CK(hipEventRecord(e1, s1));
      CK(hipStreamWaitEvent(s2, e1, 0));
      CK(hipMemcpyAsync(b, a, n * 4, hipMemcpyDeviceToDevice, s2));
      CK(hipEventRecord(e1, s2));
      CK(hipStreamWaitEvent(s1, e1, 0));
      add_one<<<n / 256, 256, 0, s1>>>(c, n);
      CK(hipEventRecord(join2, s2));
      CK(hipStreamWaitEvent(s0, join2, 0));
      break;
    case 6:
      CK(hipEventRecord(e1, s1));
      CK(hipStreamWaitEvent(s2, e1, 0));
      CK(hipMemcpyAsync(b, a, n * 4, hipMemcpyDeviceToDevice, s2));
      CK(hipEventRecord(join2, s2));
      CK(hipStreamWaitEvent(s0, join2, 0));  // s1 joined only through s2
      break;
  }
  if (cs != 6) {
    CK(hipEventRecord(join1, s1));
    CK(hipStreamWaitEvent(s0, join1, 0));
  }
  hipGraph_t graph;
  CK(hipStreamEndCapture(s0, &graph));
  fprintf(stderr, "case %d: capture ended\n", cs);
  hipGraphExec_t exe;
  CK(hipGraphInstantiate(&exe, graph, nullptr, nullptr, 0));
  CK(hipMemset(a, 0, n * 4));
  CK(hipDeviceSynchronize());
  for (int r = 0; r < 2; ++r) CK(hipGraphLaunch(exe, s0));
  CK(hipStreamSynchronize(s0));
  std::vector<float> hb(n);
  CK(hipMemcpy(hb.data(), b, n * 4, hipMemcpyDeviceToHost));
  const float want = cs == 4 ? 4.0f : (cs == 9 || cs == 10) ? 3.0f : 2.0f;
  for (size_t i = 0; i < n; ++i)
    if (hb[i] != want) {
      printf("case %d: wrong value %g at %zu (want %g)\n", cs, hb[i], i, want);
      return 1;
    }
  printf("case %d ok\n", cs);
  return 0;
}
