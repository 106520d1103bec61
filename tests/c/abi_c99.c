/* C99 consumer of include/ftar.h: the boundary needs no C++ and no HIP headers.
   Built and run by tests/test_capi.py (host-only calls, no GPU needed). */
#include <stdio.h>
#include <string.h>

#include "ftar.h"

int main(void) {
  ftar_topo_t t;
  char buf[64];
  long n;
  if (ftar_topo_parse("2,4", NULL, 8, &t) != FTAR_SUCCESS || t.nstages != 2) return 1;
  ftar_topo_format(&t, buf, sizeof buf);
  if (strcmp(buf, "2,4") != 0) return 2;
  if (ftar_topo_parse("3", NULL, 4, &t) != FTAR_ERR_INVALID_TOPO) return 3;
  if (ftar_topo_choose(8, (size_t)1 << 30, &t) != FTAR_SUCCESS) return 4;
  ftar_topo_format(&t, buf, sizeof buf);
  if (strcmp(buf, "8") != 0) return 5;
  n = ftar_schedule_json(&t, 8, 3, 1000, NULL, 0);
  if (n <= 0) return 6;
  if (ftar_dtype_size(FTAR_BFLOAT16) != 2) return 7;
  if (ftar_reduce(NULL, 0, NULL, 0, FTAR_FLOAT32, FTAR_SUM, NULL) != FTAR_ERR_INVALID_ARG) return 8;
  printf("c99 ok: %s, cost-model choice %s, schedule %ld bytes\n", ftar_version(), buf, n);
  return 0;
}
