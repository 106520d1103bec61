// ftar_benchmark — the reference's MPI benchmark harness on the MI355X path.
//
// Same command line and the same measurement as
// allreduce_over_mpi/benchmark.cpp:31-244:
//   --size N        elements (fp32), default 35            (:42, :71-77)
//   --repeat R      timed calls, default 1                  (:78-84)
//   --to-file       per-repeat times -> {tag.}{P}.{n}.{topo}.ar_test.{unix}.txt (:218-238)
//   --comm-type T   flextree|ftar (MPI_Allreduce_FT) or mpi (library MPI_Allreduce) (:90-101)
//   --tag S, --version, --check                            (:102-118)
// data[i] = i * 0.1f on every rank, in place; MPI_Barrier + MPI_Wtime around
// every call; prints "CHECK <rank>: data[9..23]" per rank and
// "DONE, average time: <avg>, min time: <min>" (:125-240).
// Extras: --device (time the device-resident entry, buffers already in HBM),
// --dump PREFIX (every rank writes its final buffer to PREFIX.<rank>.bin, raw
// fp32: the parity tests compare it with the reference's own output),
// --warmup W (untimed calls first; the reference's first call pays one-time
// setup), --no-register (host buffers: pageable copies instead of
// MPI_Allreduce_FT_register), and one JSON summary line on rank 0.
// Communicator lifecycle checks (after the timed calls):
//   --comm-cycle C    C communicators created and freed in turn, duplicates of
//                     MPI_COMM_WORLD alternating with singleton splits (MPI
//                     recycles the handles), one exact integer-valued
//                     MPI_Allreduce_FT on each;
//   --comm-threads T  T duplicates driven at once from T threads
//                     (MPI_THREAD_MULTIPLE), 3 exact calls each; on the RCCL
//                     transport only with GPU_MAX_HW_QUEUES >= 8 (T + 1), so
//                     at most T = 3 (HIP caps the queues at 32), else
//                     refused (exit 2);
//   --register-check  MPI_Allreduce_FT_register / _unregister semantics on a
//                     scratch buffer (needs a GPU: hipHostRegister).
// --check is two-sided here: the reference only flags results that are too
// LARGE (benchmark.cpp:201), so NaN/zero results pass there.
// --exact (ring or single-stage topologies, no warmup): every element must
// equal, bit for bit, the reference's fold of the P identical inputs, i.e.
// repeat times x <- x + x + ... + x (P terms, left to right in fp32: with
// identical operands every fold order of the ring, :1689-1703, and of a
// single-stage tree, :1316-1358, gives these partial sums).  Needs no dump,
// so it checks whole BASELINE-sized buckets (1 GiB per rank) in place.
// --graph (with --device): one MPI_Allreduce_FT_device call is captured into a
// HIP graph on a stream of its own (after one uncaptured call that brings the
// communicator and its buffers up, inputs restarted), and every warm-up and
// timed call replays the graph (hipGraphLaunch + hipStreamSynchronize): the
// same in-place AllReduce, so --check / --exact / --dump apply unchanged.
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "ftar_mpi.h"

static void die(int rank, const std::string& msg) {
  fprintf(stderr, "[rank %d] %s\n", rank, msg.c_str());
  MPI_Abort(MPI_COMM_WORLD, 1);
}

// A bad command line: every rank parses the same arguments, so every rank ends here and the job ends
// cleanly (MPI_Finalize, exit code 1).  MPI_Abort could kill the job before mpiexec forwarded the message.
[[noreturn]] static void usage_error(int rank, const std::string& msg) {
  fprintf(stderr, "[rank %d] %s\n", rank, msg.c_str());
  fflush(stderr);
  MPI_Finalize();
  exit(1);
}

// A failed MPI_Allreduce_FT.  The reference exit(1)s inside the call (an
// invalid FT_TOPO, mpi_mod.hpp:1471-1475); here the call returned an MPI error
// class.  An argument error fails every rank at the same call, so the ranks
// agree on it (a non-blocking allreduce, 10 s at most) and end together with
// exit code 1; a rank whose peers went on aborts the job.
[[noreturn]] static void call_failed(int rank, int P, const char* when, int rc) {
  char msg[MPI_MAX_ERROR_STRING] = "";
  int len = 0;
  MPI_Error_string(rc, msg, &len);
  const char* topo = getenv("FT_TOPO");
  fprintf(stderr, "[rank %d] allreduce failed (%s): MPI error %d: %s; FT_TOPO=%s; %s\n", rank, when, rc, msg,
          topo ? topo : "(unset)", ftar_last_error());
  fflush(stderr);
  int one = 1, failed = 0;
  MPI_Request rq;
  MPI_Iallreduce(&one, &failed, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD, &rq);
  int done = 0;
  for (int i = 0; i < 1000 && !done; ++i) {
    MPI_Test(&rq, &done, MPI_STATUS_IGNORE);
    if (!done) std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
  if (!done) MPI_Abort(MPI_COMM_WORLD, 1);
  if (rank == 0) printf("FAILED: allreduce failed on %d of %d ranks\n", failed, P);
  fflush(stdout);
  MPI_Finalize();
  exit(1);
}

int main(int argc, char** argv) {
  int provided = 0, rank = 0, P = 1;
  MPI_Init_thread(&argc, &argv, MPI_THREAD_MULTIPLE, &provided);  // benchmark.cpp:50
  MPI_Comm_size(MPI_COMM_WORLD, &P);
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);

  size_t data_len = 35;
  int repeat = 1, warmup = 0, comm_cycle = 0, comm_threads = 0;
  bool to_file = false, check = false, device = false, do_register = true, register_check = false, exact = false;
  bool graph = false;
  std::string tag, comm_type = "flextree", dump;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) usage_error(rank, "missing value for " + a);
      return argv[++i];
    };
    if (a == "--size") data_len = strtoull(next().c_str(), nullptr, 0);
    else if (a == "--repeat") repeat = atoi(next().c_str());
    else if (a == "--warmup") warmup = atoi(next().c_str());
    else if (a == "--to-file") to_file = true;
    else if (a == "--comm-type") comm_type = next();
    else if (a == "--tag") tag = next();
    else if (a == "--check") check = true;
    else if (a == "--exact") exact = true;
    else if (a == "--device") device = true;
    else if (a == "--graph") graph = true;
    else if (a == "--dump") dump = next();
    else if (a == "--no-register") do_register = false;
    else if (a == "--comm-cycle") comm_cycle = atoi(next().c_str());
    else if (a == "--comm-threads") comm_threads = atoi(next().c_str());
    else if (a == "--register-check") register_check = true;
    else if (a == "--version") {
      if (rank == 0) printf("ftar_benchmark: %s\n", ftar_version());
      MPI_Finalize();
      return 0;
    } else usage_error(rank, "unknown parameter: " + a);
  }
  if (comm_type == "ftar") comm_type = "flextree";
  if (comm_type != "flextree" && comm_type != "mpi") usage_error(rank, "unknown comm type: " + comm_type);
  if (device && comm_type == "mpi") usage_error(rank, "--device needs --comm-type flextree");
  if (graph && !device) usage_error(rank, "--graph needs --device");

  std::vector<float> data(data_len);
  const float base = 0.1f;
  for (size_t i = 0; i < data_len; ++i) data[i] = i * base;  // benchmark.cpp:125-129

  ftar_topo_t topo;
  const bool have_topo = ftar_topo_from_env(P, data_len * sizeof(float), &topo) == FTAR_SUCCESS;
  char topo_s[128] = "?";
  if (have_topo) ftar_topo_format(&topo, topo_s, sizeof topo_s);

  // the host buffer stays alive for the whole run: pin it once (RCCL-style user-buffer registration)
  const bool registered = !device && comm_type == "flextree" && do_register && data_len &&
                          MPI_Allreduce_FT_register(data.data(), data_len * sizeof(float)) == MPI_SUCCESS;
  float* dptr = nullptr;
  if (device) {
    ftar_comm_t fc;
    if (MPI_Allreduce_FT_comm(MPI_COMM_WORLD, &fc) != MPI_SUCCESS) die(rank, "communicator setup failed");
    int dev = 0;
    if (fc) ftar_comm_device(fc, &dev);
    if (hipSetDevice(dev) != hipSuccess || hipMalloc(&dptr, data_len * sizeof(float) + 4) != hipSuccess)
      die(rank, "hipMalloc failed");
    if (hipMemcpy(dptr, data.data(), data_len * sizeof(float), hipMemcpyHostToDevice) != hipSuccess)
      die(rank, "hipMemcpy failed");
  }
  MPI_Barrier(MPI_COMM_WORLD);
  if (rank == 0) {
    printf("configuration:\n  - total_peers: %d\n  - data_size: %zu\n  - repeat: %d\n  - to_file: %s\n"
           "  - check_validity: %s\n  - communication method: %s%s\n  - FlexTree topo: %s\n  - library: %s\n",
           P, data_len, repeat, to_file ? "true" : "false", check ? "true" : "false", comm_type.c_str(),
           device ? " (device-resident)" : " (host buffers)", topo_s, ftar_version());
    fflush(stdout);
  }

  hipStream_t gstream = nullptr;
  hipGraphExec_t gexec = nullptr;
  auto one_call = [&]() -> int {
    if (comm_type == "mpi") return MPI_Allreduce(MPI_IN_PLACE, data.data(), (int)data_len, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD);
    if (gexec) return hipGraphLaunch(gexec, gstream) == hipSuccess && hipStreamSynchronize(gstream) == hipSuccess
                          ? MPI_SUCCESS : MPI_ERR_OTHER;
    if (device) return MPI_Allreduce_FT_device(MPI_IN_PLACE, dptr, (int)data_len, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD, nullptr);
    return MPI_Allreduce_FT(MPI_IN_PLACE, data.data(), (int)data_len, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD);
  };
  if (graph) {  // prime uncaptured (bring-up, settings agreement, scratch growth), restart, capture one call
    if (int rc = one_call()) call_failed(rank, P, "graph priming call", rc);
    if (hipMemcpy(dptr, data.data(), data_len * sizeof(float), hipMemcpyHostToDevice) != hipSuccess)
      die(rank, "hipMemcpy failed");
    hipGraph_t g = nullptr;
    if (hipStreamCreateWithFlags(&gstream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamBeginCapture(gstream, hipStreamCaptureModeRelaxed) != hipSuccess)
      die(rank, "hipStreamBeginCapture failed");
    const int rc = MPI_Allreduce_FT_device(MPI_IN_PLACE, dptr, (int)data_len, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD,
                                           gstream);
    const hipError_t ec = hipStreamEndCapture(gstream, &g);
    if (rc != MPI_SUCCESS) call_failed(rank, P, "captured call", rc);
    if (ec != hipSuccess || hipGraphInstantiate(&gexec, g, nullptr, nullptr, 0) != hipSuccess)
      die(rank, std::string("graph capture failed: ") + hipGetErrorString(ec));
    size_t nodes = 0;
    (void)hipGraphGetNodes(g, nullptr, &nodes);
    (void)hipGraphDestroy(g);
    printf("GRAPH %d: captured %zu nodes\n", rank, nodes);
    fflush(stdout);
  }

  // warm-up calls change the data (in place, x P each); restart from i*0.1 afterwards
  for (int i = 0; i < warmup; ++i)
    if (int rc = one_call()) call_failed(rank, P, "warmup", rc);
  if (warmup) {
    for (size_t i = 0; i < data_len; ++i) data[i] = i * base;
    if (device && hipMemcpy(dptr, data.data(), data_len * sizeof(float), hipMemcpyHostToDevice) != hipSuccess)
      die(rank, "hipMemcpy failed");
  }

  std::vector<double> times;
  double sum_time = 0, min_time = 1e30;
  for (int i = 0; i < repeat; ++i) {  // benchmark.cpp:157-167
    MPI_Barrier(MPI_COMM_WORLD);
    const double t1 = MPI_Wtime();
    if (int rc = one_call()) call_failed(rank, P, "timed call", rc);
    const double t2 = MPI_Wtime();
    times.push_back(t2 - t1);
    sum_time += t2 - t1;
    min_time = std::min(min_time, t2 - t1);
  }
  if (device && hipMemcpy(data.data(), dptr, data_len * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
    die(rank, "hipMemcpy failed");

  if (!dump.empty()) {
    const std::string path = dump + "." + std::to_string(rank) + ".bin";
    std::ofstream f(path, std::ios::binary);
    f.write(reinterpret_cast<const char*>(data.data()), (std::streamsize)(data_len * sizeof(float)));
    if (!f) die(rank, "cannot write " + path);
  }

  // validity: expected i * 0.1 * P^repeat (benchmark.cpp:195-210), two-sided
  size_t bad = 0, first_bad = 0;
  if (check) {
    const double scale = std::pow((double)P, repeat);
    for (size_t i = 0; i < data_len; ++i) {
      const double exp = (double)(i * base) * scale;
      const double tol = std::max(0.01, 4.0 * P * repeat * std::fabs(exp) * 1.2e-7);
      if (!(std::fabs((double)data[i] - exp) <= tol)) {
        if (!bad) first_bad = i;
        ++bad;
      }
    }
  }
  size_t inexact = 0, first_inexact = 0;
  if (exact) {
    if (warmup) die(rank, "--exact needs --warmup 0 (the inputs are restarted after warm-up calls)");
    for (size_t i = 0; i < data_len; ++i) {
      float x = i * base;
      for (int it = 0; it < repeat; ++it) {
        float acc = x;
        for (int j = 1; j < P; ++j) acc = acc + x;
        x = acc;
      }
      if (std::memcmp(&x, &data[i], sizeof x) != 0) {
        if (!inexact) first_inexact = i;
        ++inexact;
      }
    }
  }
  for (int r = 0; r <= P; ++r) {  // ordered CHECK lines (benchmark.cpp:188-213)
    MPI_Barrier(MPI_COMM_WORLD);
    if (r == rank + 1) {
      printf("CHECK %d: ", rank);
      for (size_t i = 9; i < 24 && i < data_len; ++i) printf("%g ", data[i]);
      if (check) {
        if (!bad) printf("(test passed)");
        else printf("(test FAILED: %zu wrong, first at %zu)", bad, first_bad);
      }
      printf("\n");
      if (exact) {
        if (!inexact) printf("EXACT %d: %zu elements bit-exact\n", rank, data_len);
        else printf("EXACT %d: FAILED: %zu elements differ, first at %zu\n", rank, inexact, first_inexact);
      }
      fflush(stdout);
    }
  }
  bad += inexact;  // the exit code and the JSON line's "check" cover --exact too
  size_t bad_all = 0;
  MPI_Allreduce(&bad, &bad_all, 1, MPI_UNSIGNED_LONG, MPI_SUM, MPI_COMM_WORLD);
  double max_min = 0, max_avg = 0, avg = repeat ? sum_time / repeat : 0;
  MPI_Allreduce(&min_time, &max_min, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
  MPI_Allreduce(&avg, &max_avg, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);

  // communicator lifecycle: state released by MPI_Comm_free, fresh state under recycled handles
  int lifecycle_bad = 0;
  if (comm_cycle > 0 && comm_type == "flextree") {
    const size_t n = 4099;
    std::vector<float> buf(n);
    int reused = 0, bad_c = 0;
    MPI_Comm prev = MPI_COMM_NULL;
    for (int c = 0; c < comm_cycle; ++c) {
      MPI_Comm cc;
      const bool single = c % 2 == 1;
      if (single) MPI_Comm_split(MPI_COMM_WORLD, rank, 0, &cc);
      else MPI_Comm_dup(MPI_COMM_WORLD, &cc);
      if (c > 0 && cc == prev) ++reused;
      prev = cc;
      for (size_t i = 0; i < n; ++i) buf[i] = (float)((rank + 1) * (int)(i % 1000) + c);
      if (MPI_Allreduce_FT(MPI_IN_PLACE, buf.data(), (int)n, MPI_FLOAT, MPI_SUM, cc) != MPI_SUCCESS) ++bad_c;
      const int ranks = single ? 1 : P;
      for (size_t i = 0; i < n && !bad_c; ++i) {
        const double want = single ? (double)((rank + 1) * (int)(i % 1000) + c)
                                   : (double)P * (P + 1) / 2 * (int)(i % 1000) + (double)ranks * c;
        if ((double)buf[i] != want) ++bad_c;
      }
      MPI_Comm_free(&cc);
    }
    for (int r = 0; r <= P; ++r) {
      MPI_Barrier(MPI_COMM_WORLD);
      if (r == rank + 1) {
        printf("COMM_CYCLE %d: cycles=%d handles_reused=%d %s\n", rank, comm_cycle, reused, bad_c ? "FAILED" : "ok");
        fflush(stdout);
      }
    }
    lifecycle_bad += bad_c;
  }
  // RCCL communicators driven from several threads at once: RCCL itself deadlocks when two communicators'
  // operations reach it in different orders on different ranks -- inside ncclGroupEnd at their first
  // exchange (its lazy connection handshake; ftar's first contact now makes every connection up front), and
  // on the device once connected, when their kernels share one of the process's hardware queues (HIP's
  // default is 4 per process; with 16, two RCCL communicators in opposite orders complete: tools/rccl_order,
  // profiles/r04/rccl_order/).  So the threads run only when GPU_MAX_HW_QUEUES gives every stream of every
  // communicator a queue of its own (8 per communicator: ftar's 4, the drop-in's, RCCL's), else refused.
  const char* world_tp = "";
  if (comm_threads > 0 && comm_type == "flextree") {
    ftar_comm_t fc = nullptr;
    if (MPI_Allreduce_FT_comm(MPI_COMM_WORLD, &fc) == MPI_SUCCESS && fc) world_tp = ftar_comm_transport(fc);
  }
  const char* hwq = getenv("GPU_MAX_HW_QUEUES");
  // HIP accepts at most 32 hardware queues per process, so the RCCL transport runs at most T = 3 threads
  constexpr int kMaxHwQueues = 32;
  const int queues = hwq && *hwq ? atoi(hwq) : 4, need_queues = 8 * (comm_threads + 1);
  if (comm_threads > 0 && comm_type == "flextree" && !strcmp(world_tp, "rccl") && queues < need_queues) {
    if (rank == 0) {
      printf("COMM_THREADS refused: the RCCL transport cannot drive communicators from %d threads at once "
             "with %d hardware queues per process -- RCCL deadlocks when operations on different communicators "
             "reach the GPU in different orders on different ranks and their kernels share a queue (NCCL's "
             "rule for concurrent communicators; profiles/r04/rccl_order/); ",
             comm_threads, queues);
      if (need_queues <= kMaxHwQueues)
        printf("set GPU_MAX_HW_QUEUES >= %d, issue the calls in one agreed order, or use FTAR_MPI_TRANSPORT=ipc\n",
               need_queues);
      else
        printf("the RCCL transport supports at most %d threads (8 queues each plus the world's, HIP's limit is %d); "
               "issue the calls in one agreed order, or use FTAR_MPI_TRANSPORT=ipc\n",
               kMaxHwQueues / 8 - 1, kMaxHwQueues);
    }
    fflush(stdout);
    lifecycle_bad += 1;
  } else if (comm_threads > 0 && comm_type == "flextree") {
    if (provided < MPI_THREAD_MULTIPLE) {
      if (rank == 0) printf("COMM_THREADS skipped: MPI provides thread level %d\n", provided);
    } else {
      std::vector<MPI_Comm> comms(comm_threads);
      for (auto& cc : comms) MPI_Comm_dup(MPI_COMM_WORLD, &cc);  // same order on every rank
      std::vector<int> bad_t(comm_threads, 0);
      std::vector<std::thread> th;
      for (int t = 0; t < comm_threads; ++t)
        th.emplace_back([&, t] {
          const size_t n = 8192 + 64 * t;
          std::vector<float> b(n);
          for (int it = 0; it < 3; ++it) {
            for (size_t i = 0; i < n; ++i) b[i] = (float)((rank + 1) * (t + 1) + (int)(i % 512) + it);
            if (MPI_Allreduce_FT(MPI_IN_PLACE, b.data(), (int)n, MPI_FLOAT, MPI_SUM, comms[t]) != MPI_SUCCESS) {
              ++bad_t[t];
              return;
            }
            for (size_t i = 0; i < n; ++i) {
              const double want = (double)(t + 1) * P * (P + 1) / 2 + (double)P * ((int)(i % 512) + it);
              if ((double)b[i] != want) {
                ++bad_t[t];
                return;
              }
            }
          }
        });
      for (auto& x : th) x.join();
      for (auto& cc : comms) MPI_Comm_free(&cc);
      int bad = 0;
      for (int v : bad_t) bad += v;
      for (int r = 0; r <= P; ++r) {
        MPI_Barrier(MPI_COMM_WORLD);
        if (r == rank + 1) {
          printf("COMM_THREADS %d: threads=%d %s\n", rank, comm_threads, bad ? "FAILED" : "ok");
          fflush(stdout);
        }
      }
      lifecycle_bad += bad;
    }
  }
  if (register_check) {
    std::vector<float> buf(1 << 20, 1.0f);
    const size_t bytes = buf.size() * sizeof(float);
    int bad_r = 0;
    bad_r += MPI_Allreduce_FT_register(buf.data(), bytes) != MPI_SUCCESS;
    bad_r += MPI_Allreduce_FT_register(buf.data() + 16, 1024) != MPI_SUCCESS;  // inside a registration: no-op
    bad_r += MPI_Allreduce_FT_unregister(buf.data() + 16) != MPI_ERR_ARG;      // not a registration's start
    bad_r += MPI_Allreduce_FT(MPI_IN_PLACE, buf.data(), (int)buf.size(), MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD) !=
             MPI_SUCCESS;
    for (size_t i = 0; i < buf.size() && !bad_r; ++i) bad_r += buf[i] != (float)P;
    bad_r += MPI_Allreduce_FT_unregister(buf.data()) != MPI_SUCCESS;
    bad_r += MPI_Allreduce_FT_unregister(buf.data()) != MPI_ERR_ARG;           // already gone
    bad_r += MPI_Allreduce_FT_register(nullptr, 16) != MPI_ERR_ARG;
    printf("REGISTER_CHECK %d: %s\n", rank, bad_r ? "FAILED" : "ok");
    fflush(stdout);
    lifecycle_bad += bad_r;
  }
  int lifecycle_bad_all = 0;
  MPI_Allreduce(&lifecycle_bad, &lifecycle_bad_all, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD);

  if (gexec) (void)hipGraphExecDestroy(gexec);
  if (gstream) (void)hipStreamDestroy(gstream);
  if (device) (void)hipFree(dptr);
  if (registered) MPI_Allreduce_FT_unregister(data.data());
  MPI_Allreduce_FT_finalize();
  MPI_Finalize();

  if (rank == 0 && to_file) {  // benchmark.cpp:218-238
    std::ostringstream ss;
    if (!tag.empty()) ss << tag << ".";
    ss << P << "." << data_len << ".";
    if (comm_type == "flextree") {
      if (have_topo && !topo.ring) {
        for (int i = 0; i < topo.nstages; ++i) ss << topo.stages[i] << "-";
        ss << "+" << topo.lonely;
      } else {
        ss << "1-+0";
      }
    } else {
      ss << "mpi";
    }
    ss << ".ar_test." << time(nullptr) << ".txt";
    std::ofstream f(ss.str());
    for (double t : times) f << t << "\n";
  }
  if (rank == 0) {
    const double bytes = (double)data_len * sizeof(float);
    // a call below MPI_Wtime's resolution (a 1-rank copy) has no meaningful rate: 0 then
    const double tmin = max_min > 0 ? max_min : 1e300;
    printf("\nDONE, average time: %g, min time: %g\n", sum_time / std::max(1, repeat), min_time);
    printf("{\"harness\":\"ftar_benchmark\",\"comm_type\":\"%s\",\"resident\":\"%s\",\"P\":%d,\"count\":%zu,"
           "\"topo\":\"%s\",\"repeat\":%d,\"warmup\":%d,\"min_s\":%.6e,\"avg_s\":%.6e,\"algbw_GBps_min\":%.3f,"
           "\"busbw_GBps_min\":%.3f,\"check\":\"%s\"}\n",
           comm_type.c_str(), device ? "device" : "host", P, data_len, topo_s, repeat, warmup, max_min, max_avg,
           bytes / tmin / 1e9, P > 1 ? bytes / tmin / 1e9 * 2.0 * (P - 1) / P : bytes / tmin / 1e9,
           check || exact ? (bad_all ? "FAILED" : "passed") : "off");
  }
  return bad_all || lifecycle_bad_all ? 2 : 0;
}
