// ref_getwidth — TEST INFRASTRUCTURE ONLY (builds into oracle/_ref/).
// Our driver around the UNMODIFIED reference cost-model header
// /root/reference/cost_model/GetWidth.h: prints getWidth(P) (GetWidth.h:42-47),
// the candidate width lists the reference's cost model scores, as JSON.
#include "GetWidth.h"  // -I/root/reference/cost_model

#include <cstdio>
#include <cstdlib>

int main(int argc, char** argv) {
  int lo = argc > 1 ? atoi(argv[1]) : 1, hi = argc > 2 ? atoi(argv[2]) : 16;
  printf("{");
  for (int p = lo; p <= hi; ++p) {
    auto c = getWidth(p);
    printf("%s\"%d\":[", p == lo ? "" : ",", p);
    for (size_t i = 0; i < c.size(); ++i) {
      printf("%s[", i ? "," : "");
      for (size_t j = 0; j < c[i].size(); ++j) printf("%s%d", j ? "," : "", c[i][j]);
      printf("]");
    }
    printf("]");
  }
  printf("}\n");
  return 0;
}
