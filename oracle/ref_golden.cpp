// ============================================================================
// ref_golden — TEST INFRASTRUCTURE ONLY (builds into oracle/_ref/, never shipped).
//
// A driver of OUR OWN that includes the UNMODIFIED reference header
// /root/reference/allreduce_over_mpi/mpi_mod.hpp in its "plugin" mode
// (no STANDALONE_TEST: the header's file-static MPI_Allreduce shadows libmpi
// for this translation unit, mpi_mod.hpp:1726) and runs it under MPICH to
// produce golden vectors.  No reference source is copied into this repo; the
// header is #included from where it lies (see oracle/Makefile).
//
// Modes (all write raw little-endian bytes):
//   allreduce  --dtype D --op O --n N --seed S [--outofplace] [--repeat R]
//              [--init random|linear] --out PREFIX
//              run under `FT_TOPO=.. FT_LONELY=.. mpiexec -n P`; writes
//              PREFIX.<rank>.bin = rank's recvbuf after MPI_Allreduce.
//   schedule   --P P --topo a,b,.. --lonely L --n N
//              prints one JSON line per rank of the reference's
//              FMA_Send/FMA_Recv operations (mpi_mod.hpp:627-766).
//   reduce     --dtype D --op O --k K --n N --seed S --out FILE
//              calls FlexTree::reduce_sum / reduce_band directly.
//   arbench    --n N --repeat R   (under mpiexec, FT_TOPO set): the reference
//              MPI path timed like benchmark.cpp (C1 = P2 ring 2^20 fp32).
//   bench      --k K --n N --seconds T
//              times FlexTree::reduce_sum<float> (the cpu_baseline, kind
//              "reference"); prints one JSON line.
// Inputs come from ftar_inputs.h (splitmix64), the same generator the tests
// and the product benchmark use.
// ============================================================================
#include <mpi.h>
#include "mpi_mod.hpp"  // -I/root/reference/allreduce_over_mpi

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <omp.h>

#include "ftar_inputs.h"

using namespace FlexTree;

static const char* arg(int argc, char** argv, const char* key, const char* dflt) {
  for (int i = 1; i + 1 < argc; ++i)
    if (!strcmp(argv[i], key)) return argv[i + 1];
  return dflt;
}
static bool flag(int argc, char** argv, const char* key) {
  for (int i = 1; i < argc; ++i)
    if (!strcmp(argv[i], key)) return true;
  return false;
}

static MPI_Datatype mpi_type(int dt) {
  switch (dt) {
    case FTI_U8: return MPI_UINT8_T;
    case FTI_I8: return MPI_INT8_T;
    case FTI_U16: return MPI_UINT16_T;
    case FTI_I16: return MPI_INT16_T;
    case FTI_I32: return MPI_INT32_T;
    case FTI_I64: return MPI_INT64_T;
    case FTI_F32: return MPI_FLOAT;
    case FTI_F64: return MPI_DOUBLE;
    case FTI_BOOL: return MPI_C_BOOL;
  }
  fprintf(stderr, "dtype %d has no reference MPI type\n", dt);
  exit(2);
}

static void write_file(const std::string& path, const void* p, size_t bytes) {
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) { perror(path.c_str()); exit(3); }
  if (bytes) fwrite(p, 1, bytes, f);
  fclose(f);
}

template <class T>
static std::vector<const T*> src_array(std::vector<std::vector<uint8_t>>& in, int k) {
  std::vector<const T*> src(20 + k, nullptr);  // reduce_* read src[0..19] unconditionally
  for (int j = 0; j < k; ++j) src[j] = reinterpret_cast<const T*>(in[j].data());
  for (int j = k; j < 20; ++j) src[j] = reinterpret_cast<const T*>(in[0].data());
  return src;
}
template <class T>
static void call_sum(std::vector<std::vector<uint8_t>>& in, std::vector<uint8_t>& out, int k, size_t n) {
  auto src = src_array<T>(in, k);
  reduce_sum<T>(src.data(), reinterpret_cast<T*>(out.data()), k, n);
}
template <class T>
static void call_band(std::vector<std::vector<uint8_t>>& in, std::vector<uint8_t>& out, int k, size_t n) {
  auto src = src_array<T>(in, k);
  reduce_band<T>(src.data(), reinterpret_cast<T*>(out.data()), k, n);
}
template <class T>
static void call_reduce(int op, std::vector<std::vector<uint8_t>>& in, std::vector<uint8_t>& out, int k, size_t n) {
  if (op == 0) call_sum<T>(in, out, k, n);
  else call_band<T>(in, out, k, n);
}

static int mode_reduce(int argc, char** argv) {
  int dt = atoi(arg(argc, argv, "--dtype", "6"));
  int op = atoi(arg(argc, argv, "--op", "0"));
  int k = atoi(arg(argc, argv, "--k", "2"));
  size_t n = strtoull(arg(argc, argv, "--n", "16"), 0, 10);
  uint64_t seed = strtoull(arg(argc, argv, "--seed", "1"), 0, 10);
  std::string out = arg(argc, argv, "--out", "reduce.bin");
  size_t esz = fti_dtype_size(dt);
  std::vector<std::vector<uint8_t>> in(k);
  for (int j = 0; j < k; ++j) {
    in[j].resize(n * esz + 8);
    fti_fill(dt, seed, (uint64_t)j, in[j].data(), n);
  }
  std::vector<uint8_t> o(n * esz + 8, 0xA5);
  switch (dt) {
    case FTI_U8: call_reduce<uint8_t>(op, in, o, k, n); break;
    case FTI_I8: call_reduce<int8_t>(op, in, o, k, n); break;
    case FTI_U16: call_reduce<uint16_t>(op, in, o, k, n); break;
    case FTI_I16: call_reduce<int16_t>(op, in, o, k, n); break;
    case FTI_I32: call_reduce<int32_t>(op, in, o, k, n); break;
    case FTI_I64: call_reduce<int64_t>(op, in, o, k, n); break;
    case FTI_F32: if (op) return 4; call_sum<float>(in, o, k, n); break;
    case FTI_F64: if (op) return 4; call_sum<double>(in, o, k, n); break;
    case FTI_BOOL: if (op) return 4; call_sum<bool>(in, o, k, n); break;
    default: return 4;
  }
  write_file(out, o.data(), n * esz);
  return 0;
}

static int mode_allreduce(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  int rank, P;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &P);
  int dt = atoi(arg(argc, argv, "--dtype", "6"));
  int op = atoi(arg(argc, argv, "--op", "0"));
  size_t n = strtoull(arg(argc, argv, "--n", "16"), 0, 10);
  uint64_t seed = strtoull(arg(argc, argv, "--seed", "1"), 0, 10);
  bool oop = flag(argc, argv, "--outofplace");
  int repeat = atoi(arg(argc, argv, "--repeat", "1"));
  std::string out = arg(argc, argv, "--out", "ar");
  size_t esz = fti_dtype_size(dt);
  std::vector<uint8_t> in(n * esz + 8), rb(n * esz + 8, 0xA5);
  if (!strcmp(arg(argc, argv, "--init", "random"), "linear") && dt == FTI_F32) {
    // benchmark.cpp:125-129: data[i] = i * 0.1f on every rank
    const float base = 0.1;
    for (size_t i = 0; i < n; ++i) reinterpret_cast<float*>(in.data())[i] = i * base;
  } else {
    fti_fill(dt, seed, (uint64_t)rank, in.data(), n);
  }
  for (int it = 0; it < repeat; ++it) {
    if (oop) {
      MPI_Allreduce(in.data(), rb.data(), (int)n, mpi_type(dt), op ? MPI_BAND : MPI_SUM, MPI_COMM_WORLD);
      if (it + 1 < repeat) memcpy(in.data(), rb.data(), n * esz);
    } else {
      if (it == 0) memcpy(rb.data(), in.data(), n * esz);
      MPI_Allreduce(MPI_IN_PLACE, rb.data(), (int)n, mpi_type(dt), op ? MPI_BAND : MPI_SUM, MPI_COMM_WORLD);
    }
  }
  write_file(out + "." + std::to_string(rank) + ".bin", rb.data(), n * esz);
  MPI_Finalize();
  return 0;
}

// benchmark.cpp:125-167 semantics with the reference's own MPI_Allreduce_FT:
// data[i] = i*0.1f, in place, MPI_Barrier + MPI_Wtime around each call.
static int mode_arbench(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  int rank, P;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &P);
  size_t n = strtoull(arg(argc, argv, "--n", "1048576"), 0, 10);
  int repeat = atoi(arg(argc, argv, "--repeat", "20"));
  std::vector<float> data(n);
  const float base = 0.1;
  for (size_t i = 0; i < n; ++i) data[i] = i * base;
  double sum = 0, mn = 1e30, first = 0;
  for (int it = 0; it < repeat; ++it) {
    MPI_Barrier(MPI_COMM_WORLD);
    double t1 = MPI_Wtime();
    MPI_Allreduce(MPI_IN_PLACE, data.data(), (int)n, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD);
    double t2 = MPI_Wtime();
    if (it == 0) first = t2 - t1;
    else sum += t2 - t1;  // mean excludes the first call (OMP team + buffer setup)
    mn = std::min(mn, t2 - t1);
  }
  double mx_min = 0, mean = repeat > 1 ? sum / (repeat - 1) : first, mx_mean = 0;
  MPI_Reduce(&mn, &mx_min, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
  MPI_Reduce(&mean, &mx_mean, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
  if (rank == 0) {
    const char* topo = getenv("FT_TOPO");
    printf("{\"kind\":\"reference\",\"P\":%d,\"n\":%zu,\"topo\":\"%s\",\"repeat\":%d,\"min_s\":%.6e,"
           "\"mean_s\":%.6e,\"first_s\":%.6e,\"algbw_GBps_min\":%.4f,\"threads_per_rank\":14}\n",
           P, n, topo ? topo : "", repeat, mx_min, mx_mean, first, n * 4.0 / mx_min / 1e9);
  }
  MPI_Finalize();
  return 0;
}

static std::string json_ops(const std::vector<std::vector<FMA_Operation>>& v) {
  std::string s = "[";
  for (size_t i = 0; i < v.size(); ++i) {
    s += i ? ",[" : "[";
    for (size_t j = 0; j < v[i].size(); ++j) {
      const FMA_Operation& m = v[i][j];
      s += (j ? ",{" : "{");
      s += "\"peer\":" + std::to_string(m.peer) + ",\"src\":" + (m.from_src ? "1" : "0") + ",\"r\":[";
      for (size_t q = 0; q < m.ranges.size(); ++q) {
        s += (q ? ",[" : "[") + std::to_string(m.ranges[q].addr) + "," + std::to_string(m.ranges[q].len) + "," +
             std::to_string(m.ranges[q].actual_addr) + "]";
      }
      s += "]}";
    }
    s += "]";
  }
  return s + "]";
}

static int mode_schedule(int argc, char** argv) {
  size_t P = strtoull(arg(argc, argv, "--P", "4"), 0, 10);
  size_t L = strtoull(arg(argc, argv, "--lonely", "0"), 0, 10);
  size_t n = strtoull(arg(argc, argv, "--n", "16"), 0, 10);
  std::string topo = arg(argc, argv, "--topo", "4");
  std::vector<size_t> st;
  size_t pos = 0;
  while (pos <= topo.size()) {
    size_t c = topo.find(',', pos);
    if (c == std::string::npos) c = topo.size();
    if (c > pos) st.push_back(strtoull(topo.substr(pos, c - pos).c_str(), 0, 10));
    pos = c + 1;
  }
  for (size_t r = 0; r < P; ++r) {
    Send_Operations so(P, L, r, st);
    Recv_Operations ro(P, L, r, st);
    so.generate();
    ro.generate();
    FMA_Send_Operations fs(&so, &ro, P, n);
    FMA_Recv_Operations fr(&so, &ro, P, n);
    fs.generate();
    fr.generate();
    printf("{\"rank\":%zu,\"send\":%s,\"send_lonely\":%s,\"recv\":%s,\"recv_lonely\":%s}\n", r,
           json_ops(fs.FMA_ops).c_str(), json_ops(fs.FMA_lonely_ops).c_str(), json_ops(fr.FMA_ops).c_str(),
           json_ops(fr.FMA_lonely_ops).c_str());
  }
  return 0;
}

// --sets S: S disjoint (k sources + destination) buffer sets used in turn, one per call (S = 1: the same
// buffers every call, warm in the host's caches as far as they fit; S >= 2: each call finds its buffers
// evicted by the calls before it, the regime bench.py's GPU line runs in)
static int mode_bench(int argc, char** argv) {
  int k = atoi(arg(argc, argv, "--k", "2"));
  size_t n = strtoull(arg(argc, argv, "--n", "67108864"), 0, 10);
  double seconds = atof(arg(argc, argv, "--seconds", "10"));
  int sets = atoi(arg(argc, argv, "--sets", "1"));
  if (sets < 1) sets = 1;
  std::vector<std::vector<std::vector<float>>> in(sets, std::vector<std::vector<float>>(k, std::vector<float>(n)));
  for (int s = 0; s < sets; ++s)
    for (int j = 0; j < k; ++j) fti_fill(FTI_F32, 0x5EED, (uint64_t)j, in[s][j].data(), n);
  std::vector<std::vector<float>> outs(sets, std::vector<float>(n));
  std::vector<std::vector<const float*>> srcs(sets, std::vector<const float*>(20, in[0][0].data()));
  for (int s = 0; s < sets; ++s)
    for (int j = 0; j < k; ++j) srcs[s][j] = in[s][j].data();
  for (int s = 0; s < sets; ++s)
    reduce_sum<float>(srcs[s].data(), outs[s].data(), k, n);  // warm-up: OMP team start + first touch
  std::vector<float>& out = outs[0];
  int iters = 0;
  double best = 1e30, total = 0;
  std::vector<double> times;
  auto t_end = std::chrono::steady_clock::now() + std::chrono::duration<double>(seconds);
  do {
    const int s = iters % sets;
    auto t0 = std::chrono::steady_clock::now();
    reduce_sum<float>(srcs[s].data(), outs[s].data(), k, n);
    auto t1 = std::chrono::steady_clock::now();
    double dt = std::chrono::duration<double>(t1 - t0).count();
    best = dt < best ? dt : best;
    total += dt;
    times.push_back(dt);
    ++iters;
  } while (std::chrono::steady_clock::now() < t_end);
  std::sort(times.begin(), times.end());
  const double median = times[times.size() / 2];
  double bytes = (double)(k + 1) * n * sizeof(float);
  printf("{\"kind\":\"reference\",\"k\":%d,\"n\":%zu,\"sets\":%d,\"iters\":%d,\"best_s\":%.6f,\"mean_s\":%.6f,"
         "\"median_s\":%.6f,\"GBps_best\":%.3f,\"GBps_mean\":%.3f,\"GBps_median\":%.3f,\"threads\":%d,"
         "\"checksum\":%.9g}\n",
         k, n, sets, iters, best, total / iters, median, bytes / best / 1e9, bytes / (total / iters) / 1e9,
         bytes / median / 1e9, 14 /* PARALLEL_THREAD, mpi_mod.hpp:820 */, (double)out[n / 3]);
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: ref_golden allreduce|schedule|reduce|bench ...\n");
    return 1;
  }
  std::string m = argv[1];
  if (m == "allreduce") return mode_allreduce(argc, argv);
  if (m == "schedule") return mode_schedule(argc, argv);
  if (m == "reduce") return mode_reduce(argc, argv);
  if (m == "bench") return mode_bench(argc, argv);
  if (m == "arbench") return mode_arbench(argc, argv);
  fprintf(stderr, "unknown mode %s\n", m.c_str());
  return 1;
}
