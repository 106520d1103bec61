// Host-only stress of the plan compiler (schedule.cpp) under AddressSanitizer
// and UndefinedBehaviorSanitizer (tests/test_sanitize.py builds and runs it):
// every ordered factorization of P = 2..max_base (plus lonely ranks 1..3 and
// the ring), sizes 0 / 1 / P-1 / ragged / large, every data-movement form, all
// ranks; malformed ftar_topo_t values must be rejected without touching memory
// they do not own.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ftar_internal.h"

namespace ftar {
void set_error(const std::string&, const char*, int) {}  // schedule.cpp needs no error text here
}  // namespace ftar

static void factorizations(int n, std::vector<int>& cur, std::vector<std::vector<int>>& out) {
  if (n == 1) {
    if (!cur.empty()) out.push_back(cur);
    return;
  }
  for (int f = 2; f <= n; ++f)
    if (n % f == 0) {
      cur.push_back(f);
      factorizations(n / f, cur, out);
      cur.pop_back();
    }
}

int main(int argc, char** argv) {
  const int max_base = argc > 1 ? std::atoi(argv[1]) : 24;
  long plans = 0, worlds = 0, rejected = 0;
  const ftar::Form forms[4] = {{FTAR_AG_STAGES, FTAR_RS_STAGES}, {FTAR_AG_DIRECT, FTAR_RS_DIRECT},
                               {FTAR_AG_COLLECTIVE, FTAR_RS_DIRECT}, {FTAR_AG_COLLECTIVE, FTAR_RS_STAGES}};
  for (int base = 2; base <= max_base; ++base) {
    std::vector<int> cur;
    std::vector<std::vector<int>> fs;
    factorizations(base, cur, fs);
    fs.push_back({1});  // ring marker
    for (auto& f : fs) {
      for (int lonely = 0; lonely <= 3; ++lonely) {
        const bool ring = f.size() == 1 && f[0] == 1;
        if (ring && lonely) continue;
        const int P = ring ? base : base + lonely;
        if (f.size() > FTAR_MAX_STAGES) continue;
        ftar_topo_t t{};
        t.nstages = (int)f.size();
        for (size_t i = 0; i < f.size(); ++i) t.stages[i] = f[i];
        t.lonely = lonely;
        t.ring = ring;
        ftar::Topology topo;
        if (ftar::to_topology(&t, P, &topo) != FTAR_SUCCESS) {
          ++rejected;
          continue;
        }
        for (size_t count : {size_t(0), size_t(1), size_t(P - 1), size_t(P) * 7 + 3, size_t(1) << 20}) {
          for (const auto& form : forms) {
            if (ftar::check_world(topo, P, count, form) != FTAR_SUCCESS) {
              ++rejected;
              continue;
            }
            ++worlds;
            for (int r = 0; r < P; ++r) {
              ftar::Plan p;
              if (ftar::build_plan(topo, P, r, count, &p, form) != FTAR_SUCCESS) return 2;
              std::string js = p.json();
              if (js.empty()) return 3;
              if (!ring) {
                std::string sj;
                if (ftar::schedule_json(topo, P, r, count, &sj) != FTAR_SUCCESS) return 4;
              }
              ++plans;
            }
          }
        }
      }
    }
  }
  // malformed inputs: rejected, never read out of bounds
  ftar_topo_t bad{};
  ftar::Topology out;
  const int nst[] = {0, -1, FTAR_MAX_STAGES + 1, 1 << 30};
  for (int n : nst) {
    bad.nstages = n;
    if (ftar::to_topology(&bad, 8, &out) == FTAR_SUCCESS && n > FTAR_MAX_STAGES) return 5;
  }
  bad.nstages = 2;
  bad.stages[0] = 0;
  bad.stages[1] = -3;
  if (ftar::to_topology(&bad, 8, &out) == FTAR_SUCCESS) return 6;
  bad.stages[0] = 1 << 30;
  bad.stages[1] = 1 << 30;
  if (ftar::to_topology(&bad, 8, &out) == FTAR_SUCCESS) return 7;
  bad.stages[0] = 2;
  bad.stages[1] = 2;
  bad.lonely = -1;
  if (ftar::to_topology(&bad, 8, &out) == FTAR_SUCCESS) return 8;
  std::printf("{\"plans\": %ld, \"worlds\": %ld, \"rejected\": %ld}\n", plans, worlds, rejected);
  return 0;
}
