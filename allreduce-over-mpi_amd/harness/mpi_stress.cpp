// Random calls through the MPI drop-in (libftar_mpi.so: MPI_Allreduce_FT and MPI_Allreduce_FT_device), every
// result checked: MPI datatypes of the reference (mpi_mod.hpp:1363-1412) with MPI_SUM and MPI_BAND, empty and
// ragged counts, FT_TOPO / FT_LONELY set per call in the environment (read on every call, as get_stages is,
// mpi_mod.hpp:1732), MPI_IN_PLACE and separate buffers, host buffers (registered or pageable) and device
// buffers, and calls on duplicated communicators freed again.  Every rank draws the same sequence.  Inputs are
// small integers, so the expected value of every element is the plain sum (or AND) in any order.
//
//   mpiexec -n P ftar_mpi_stress CALLS SEED      (FTAR_MPI_TRANSPORT=ipc: one-round layouts only)
#include <hip/hip_runtime.h>
#include <mpi.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "ftar_mpi.h"

namespace {

struct Ty {
  MPI_Datatype mpi;
  size_t size;
  int kind;  // 0 float, 1 double, 2 signed int, 3 unsigned int
  const char* name;
};

long value(size_t i, int r, bool band) {
  return band ? (long)((i * 2654435761u + (size_t)r * 40503u) & 0x7fffffff) : (long)((i * 7 + r * 13 + (i >> 9)) % 17) - 8;
}

void put(const Ty& t, uint8_t* p, long v) {
  switch (t.size * 10 + t.kind) {
    case 40: { float f = (float)v; memcpy(p, &f, 4); break; }
    case 81: { double f = (double)v; memcpy(p, &f, 8); break; }
    case 42: { int32_t x = (int32_t)v; memcpy(p, &x, 4); break; }
    case 82: { int64_t x = v; memcpy(p, &x, 8); break; }
    case 22: { int16_t x = (int16_t)v; memcpy(p, &x, 2); break; }
    case 13: *p = (uint8_t)v; break;
    default: abort();
  }
}

// the expected element: sum (wrapping for integers) or AND over the ranks, in the element type
void expected(const Ty& t, uint8_t* p, size_t i, int P, bool band) {
  if (t.kind <= 1) {
    double s = 0;
    for (int r = 0; r < P; ++r) s += (double)value(i, r, false);
    put(t, p, (long)s);
    return;
  }
  uint64_t acc = band ? ~uint64_t(0) : 0;
  for (int r = 0; r < P; ++r) {
    const uint64_t v = (uint64_t)value(i, r, band);
    acc = band ? (acc & v) : acc + v;
  }
  put(t, p, (long)acc);  // truncated to the type: the wrapped sum / the AND
}

[[noreturn]] void die(int rank, const std::string& what) {
  fprintf(stderr, "FAIL rank %d: %s\n", rank, what.c_str());
  fflush(stderr);
  MPI_Abort(MPI_COMM_WORLD, 1);
  _Exit(1);
}

}  // namespace

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  int rank = 0, P = 1;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &P);
  const long calls = argc > 1 ? atol(argv[1]) : 200;
  const unsigned long seed = argc > 2 ? strtoul(argv[2], nullptr, 0) : 1;
  const char* tr = getenv("FTAR_MPI_TRANSPORT");
  const bool one_round_only = tr && !strcmp(tr, "ipc");
  const Ty types[] = {{MPI_FLOAT, 4, 0, "float"},     {MPI_DOUBLE, 8, 1, "double"}, {MPI_INT32_T, 4, 2, "int32"},
                      {MPI_INT64_T, 8, 2, "int64"},   {MPI_INT16_T, 2, 2, "int16"}, {MPI_UINT8_T, 1, 3, "uint8"}};
  // FT_TOPO / FT_LONELY layouts valid at P (lonely ones need the RCCL transport's staged rounds)
  std::vector<std::pair<std::string, std::string>> lay = {{"1", "0"}, {std::to_string(P), "0"}};
  if (P == 4) lay.push_back({"2,2", "0"});
  if (P == 6) lay.insert(lay.end(), {{"2,3", "0"}, {"3,2", "0"}});
  if (P == 8) lay.insert(lay.end(), {{"2,4", "0"}, {"2,2,2", "0"}});
  if (!one_round_only) {
    if (P == 5) lay.push_back({"2,2", "1"});
    if (P == 6) lay.push_back({"2,2", "2"});
    if (P == 8) lay.push_back({"3,2", "2"});
  }
  std::mt19937_64 rng(seed);
  long checked = 0, on_dups = 0, device_calls = 0, registered = 0;
  for (long call = 0; call < calls; ++call) {
    const Ty& t = types[rng() % 6];
    const bool band = t.kind >= 2 && rng() % 3 == 0;
    const size_t counts[] = {0, 1, (size_t)P - 1, (size_t)P + 1, 1000 + rng() % 5000, 100000 + rng() % 200000};
    const size_t n = counts[rng() % 6];
    const auto& L = lay[rng() % lay.size()];
    const bool in_place = rng() % 2 == 0;
    const bool device = rng() % 4 == 0;
    const bool reg = !device && rng() % 3 == 0;
    const bool dup = rng() % 10 == 0;
    setenv("FT_TOPO", L.first.c_str(), 1);
    setenv("FT_LONELY", L.second.c_str(), 1);
    const size_t bytes = n * t.size;
    std::vector<uint8_t> in(bytes), out(bytes, 0x5a), want(bytes);
    for (size_t i = 0; i < n; ++i) {
      put(t, &in[i * t.size], value(i, rank, band));
      expected(t, &want[i * t.size], i, P, band);
    }
    MPI_Comm comm = MPI_COMM_WORLD;
    if (dup) {
      MPI_Comm_dup(MPI_COMM_WORLD, &comm);
      ++on_dups;
    }
    const MPI_Op op = band ? MPI_BAND : MPI_SUM;
    char what[256];
    snprintf(what, sizeof what, "call %ld: %s %s n=%zu FT_TOPO=%s FT_LONELY=%s in_place=%d device=%d reg=%d dup=%d",
             call, t.name, band ? "band" : "sum", n, L.first.c_str(), L.second.c_str(), in_place, device, reg, dup);
    int rc;
    std::vector<uint8_t> got;
    if (device) {
      void *a = nullptr, *b = nullptr;
      if (hipMalloc(&a, bytes ? bytes : 1) != hipSuccess || hipMalloc(&b, bytes ? bytes : 1) != hipSuccess)
        die(rank, "hipMalloc");
      if (bytes && hipMemcpy(a, in.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) die(rank, "hipMemcpy");
      rc = MPI_Allreduce_FT_device(in_place ? MPI_IN_PLACE : a, in_place ? a : b, (int)n, t.mpi, op, comm, nullptr);
      got.resize(bytes);
      if (bytes && hipMemcpy(got.data(), in_place ? a : b, bytes, hipMemcpyDeviceToHost) != hipSuccess)
        die(rank, "hipMemcpy back");
      if (hipFree(a) != hipSuccess || hipFree(b) != hipSuccess) die(rank, "hipFree");
      ++device_calls;
    } else {
      uint8_t* buf = in_place ? in.data() : out.data();
      if (reg && bytes) {
        if (MPI_Allreduce_FT_register(in.data(), bytes) != MPI_SUCCESS) die(rank, std::string(what) + ": register");
        if (!in_place && MPI_Allreduce_FT_register(out.data(), bytes) != MPI_SUCCESS)
          die(rank, std::string(what) + ": register out");
        ++registered;
      }
      rc = MPI_Allreduce_FT(in_place ? MPI_IN_PLACE : in.data(), buf, (int)n, t.mpi, op, comm);
      if (reg && bytes) {
        MPI_Allreduce_FT_unregister(in.data());
        if (!in_place) MPI_Allreduce_FT_unregister(out.data());
      }
      got.assign(buf, buf + bytes);
    }
    if (rc != MPI_SUCCESS) die(rank, std::string(what) + ": returned " + std::to_string(rc));
    if (got != want) {
      size_t i = 0;
      while (i < bytes && got[i] == want[i]) ++i;
      die(rank, std::string(what) + ": differs at byte " + std::to_string(i));
    }
    ++checked;
    if (dup) MPI_Comm_free(&comm);
    if (rank == 0 && (call + 1) % 50 == 0) {
      printf("progress: %ld calls\n", call + 1);
      fflush(stdout);
    }
  }
  printf("{\"rank\": %d, \"checked\": %ld, \"device\": %ld, \"registered\": %ld, \"on_dups\": %ld}\n", rank, checked,
         device_calls, registered, on_dups);
  fflush(stdout);
  MPI_Allreduce_FT_finalize();
  MPI_Finalize();
  return 0;
}
