// replay — re-issues, from ONE thread, the stream/event/copy/kernel calls a
// capture made (an op file extracted from an AMD_LOG_LEVEL=4 log by
// tools/capture/extract_ops.py), with stand-in streams, events, buffers and
// a dummy kernel.  A crash here reproduces the hipStreamEndCapture crash
// outside ftar; dropping ops (argv[2] = kinds to drop, e.g. "m" = memcpys,
// "k" = kernels) bisects it.
//   ops: B s | R e s | W s e | M s | K s | E s
// argv[3] = k: stop after the k-th op, join every stream used so far into the
// origin stream and end the capture there (the shortest crashing prefix).
// argv[4] = i: skip the i-th op (which ops the crash needs).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "line %d: %s: %s\n", lineno, #x, hipGetErrorString(e_));            \
      exit(2);                                                                             \
    }                                                                                      \
  } while (0)

__global__ void touch(float* p) { p[threadIdx.x] += 1.0f; }

int main(int argc, char** argv) {
  std::ifstream in(argv[1]);
  const std::string drop = argc > 2 ? argv[2] : "";
  const int stop_after = argc > 3 ? atoi(argv[3]) : -1;
  const int skip = argc > 4 ? atoi(argv[4]) : -1;
  std::string origin;
  std::map<std::string, hipStream_t> streams;
  std::map<std::string, hipEvent_t> events;
  int lineno = 0;
  float *a, *b;
  CK(hipMalloc(&a, 1 << 20));
  CK(hipMalloc(&b, 1 << 20));
  auto S = [&](const std::string& k) {
    if (!streams.count(k)) CK(hipStreamCreateWithFlags(&streams[k], hipStreamNonBlocking));
    return streams[k];
  };
  auto E = [&](const std::string& k) {
    if (!events.count(k)) CK(hipEventCreateWithFlags(&events[k], hipEventDisableTiming));
    return events[k];
  };
  std::string line;
  int n = 0;
  while (std::getline(in, line)) {
    ++lineno;
    std::istringstream ls(line);
    std::string op, x, y;
    ls >> op >> x >> y;
    if (!op.empty() && drop.find(op[0] | 0x20) != std::string::npos && op != "B" && op != "E") continue;
    if (op != "B" && op != "E" && stop_after >= 0 && n >= stop_after) {
      // join everything used so far into the origin and end there
      for (auto& kv : streams) {
        if (kv.first == origin) continue;
        hipEvent_t j;
        CK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
        CK(hipEventRecord(j, kv.second));
        CK(hipStreamWaitEvent(streams[origin], j, 0));
      }
      op = "E";
      x = origin;
    }
    if (op != "B" && op != "E" && n == skip) {
      ++n;
      continue;
    }
    if (op == "B") {
      origin = x;
      CK(hipStreamBeginCapture(S(x), hipStreamCaptureModeRelaxed));
    }
    else if (op == "R") CK(hipEventRecord(E(x), S(y)));
    else if (op == "W") CK(hipStreamWaitEvent(S(x), E(y), 0));
    else if (op == "M") CK(hipMemcpyAsync(b, a, 256, hipMemcpyDeviceToDevice, S(x)));
    else if (op == "K") touch<<<1, 64, 0, S(x)>>>(a);
    else if (op == "E") {
      hipGraph_t g;
      fprintf(stderr, "replay: %d ops, ending the capture\n", n);
      CK(hipStreamEndCapture(S(x), &g));
      size_t nodes = 0;
      CK(hipGraphGetNodes(g, nullptr, &nodes));
      printf("replay ok: %zu nodes (dropped '%s')\n", nodes, drop.c_str());
      return 0;
    }
    ++n;
  }
  fprintf(stderr, "no end of capture in the op file\n");
  return 1;
}
