// ref_costmodel — TEST INFRASTRUCTURE ONLY (builds into oracle/_ref/).
// Our driver around the UNMODIFIED reference cost-model headers
// /root/reference/cost_model/GetWidth.h + CostModel.h: for every P and chunk
// size asked for, runs CostModel(getWidth(P), P, chunk) (CostModel.h:82-120,
// as cost_model/main.cpp:22-23 does) with its console output captured, and
// prints one JSON object per (P, chunk): the candidate lists, the per-candidate
// "single cost" lines in order, and the printed argmin and its cost.
// Built at -O0 like the reference's own CMakeLists.txt (no optimisation level
// set): the model reads an uninitialised `cost` on its first candidate
// (CostModel.h:89), which -O0 happens to leave ~0 and -O2 turns into a stack
// smash at P = 1; P = 1 (an empty width list, no return, CostModel.h:40-78)
// is never asked for.
#include <iostream>
#include <sstream>
#include <string>
#include <vector>
using namespace std;
#include "GetWidth.h"   // -I/root/reference/cost_model
#include "CostModel.h"

#include <cstdio>
#include <cstdlib>

int main(int argc, char** argv) {
  const int lo = argc > 1 ? atoi(argv[1]) : 1, hi = argc > 2 ? atoi(argv[2]) : 24;
  std::vector<double> chunks;
  for (int i = 3; i < argc; ++i) chunks.push_back(atof(argv[i]));
  if (chunks.empty()) chunks.push_back(100.0);  // cost_model/main.cpp:23
  for (double ch : chunks)
    for (int p = lo; p <= hi; ++p) {
      auto cands = getWidth(p);
      std::ostringstream cap;
      cout.precision(17);  // the stream's state, not the reference's code: full doubles in the captured lines
      std::streambuf* old = cout.rdbuf(cap.rdbuf());
      CostModel(cands, p, ch);
      cout.rdbuf(old);
      std::vector<std::string> costs;
      std::string chosen, best;
      std::istringstream in(cap.str());
      std::string line;
      const std::string k1 = "the single cost should be: ", k2 = "total nodes should be: ";
      while (std::getline(in, line)) {
        if (line.rfind(k1, 0) == 0) costs.push_back(line.substr(k1.size()));
        const size_t at = line.find(k2);
        if (at != std::string::npos) {
          if (line.find("tree structure") != std::string::npos) chosen = line.substr(at + k2.size());
          else best = line.substr(at + k2.size());
        }
      }
      printf("{\"P\":%d,\"chunk\":%g,\"candidates\":[", p, ch);
      for (size_t i = 0; i < cands.size(); ++i) {
        printf("%s[", i ? "," : "");
        for (size_t j = 0; j < cands[i].size(); ++j) printf("%s%d", j ? "," : "", cands[i][j]);
        printf("]");
      }
      printf("],\"costs\":[");
      for (size_t i = 0; i < costs.size(); ++i) printf("%s\"%s\"", i ? "," : "", costs[i].c_str());
      printf("],\"chosen\":\"%s\",\"cost\":\"%s\"}\n", chosen.c_str(), best.c_str());
    }
  return 0;
}
