/* The MPI drop-in's type/op mapping against the reference's handle_reduce dispatch
   (allreduce_over_mpi/mpi_mod.hpp:1363-1412): every MPI datatype the reference reduces maps to the ftar
   dtype of the same width and signedness, BAND is accepted, anything else is MPI_ERR_TYPE / MPI_ERR_OP, and
   MPI_Allreduce_FT on a 1-rank communicator copies (mpi_mod.hpp:1739-1746) for every type.
   FT_TOPO / FT_LONELY are read on every call (get_stages, mpi_mod.hpp:1732): a value invalid for the
   communicator's size is MPI_ERR_ARG even on one rank (the reference: "invalid FT_TOPO", exit(1),
   :1471-1475), and a change between two calls takes effect at the next call.
   Built and run by tests/test_capi.py under mpiexec -n 1 (no GPU needed). */
#define _POSIX_C_SOURCE 200112L /* setenv / unsetenv under -std=c99 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ftar_mpi.h"

static int check(MPI_Datatype d, ftar_dtype_t want, const char* name) {
  ftar_dtype_t got;
  if (ftar_mpi_dtype(d, &got) != MPI_SUCCESS || got != want) {
    printf("%s: wrong mapping\n", name);
    return 1;
  }
  return 0;
}

int main(int argc, char** argv) {
  int bad = 0, i;
  ftar_dtype_t dt;
  ftar_op_t op;
  unsigned char in[64], out[64];
  MPI_Init(&argc, &argv);
  bad += check(MPI_UINT8_T, FTAR_UINT8, "MPI_UINT8_T");
  bad += check(MPI_INT8_T, FTAR_INT8, "MPI_INT8_T");
  bad += check(MPI_UINT16_T, FTAR_UINT16, "MPI_UINT16_T");
  bad += check(MPI_INT16_T, FTAR_INT16, "MPI_INT16_T");
  bad += check(MPI_INT32_T, FTAR_INT32, "MPI_INT32_T");
  bad += check(MPI_INT64_T, FTAR_INT64, "MPI_INT64_T");
  bad += check(MPI_LONG_LONG, FTAR_INT64, "MPI_LONG_LONG");
  bad += check(MPI_FLOAT, FTAR_FLOAT32, "MPI_FLOAT");
  bad += check(MPI_DOUBLE, FTAR_FLOAT64, "MPI_DOUBLE");
  bad += check(MPI_C_BOOL, FTAR_BOOL, "MPI_C_BOOL");
  bad += ftar_mpi_dtype(MPI_LONG_DOUBLE, &dt) != MPI_ERR_TYPE;
  bad += ftar_mpi_dtype(MPI_CHAR, &dt) != MPI_ERR_TYPE;
  bad += ftar_mpi_op(MPI_SUM, &op) != MPI_SUCCESS || op != FTAR_SUM;
  bad += ftar_mpi_op(MPI_BAND, &op) != MPI_SUCCESS || op != FTAR_BAND;
  bad += ftar_mpi_op(MPI_MAX, &op) != MPI_ERR_OP;
  for (i = 0; i < 64; ++i) in[i] = (unsigned char)(i * 7 + 1);
  memset(out, 0, sizeof out);
  bad += MPI_Allreduce_FT(in, out, 16, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD) != MPI_SUCCESS;
  bad += memcmp(in, out, 64) != 0;
  memset(out, 0, sizeof out);
  bad += MPI_Allreduce_FT(in, out, 8, MPI_INT64_T, MPI_BAND, MPI_COMM_WORLD) != MPI_SUCCESS;
  bad += memcmp(in, out, 64) != 0;
  bad += MPI_Allreduce_FT(in, out, 4, MPI_CHAR, MPI_SUM, MPI_COMM_WORLD) != MPI_ERR_TYPE;
  bad += MPI_Allreduce_FT(in, out, 4, MPI_FLOAT, MPI_MAX, MPI_COMM_WORLD) != MPI_ERR_OP;
  bad += MPI_Allreduce_FT(in, NULL, 4, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD) != MPI_ERR_ARG;
  bad += MPI_Allreduce_FT(NULL, NULL, 0, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD) != MPI_SUCCESS;
  bad += MPI_Allreduce_FT(in, out, 4, MPI_FLOAT, MPI_SUM, MPI_COMM_NULL) != MPI_ERR_COMM;
  /* FT_TOPO per call */
  {
    static const char* bad_topos[] = {"3", "2,2", "0", "2,x", "-1", "abc"};
    size_t t;
    for (t = 0; t < sizeof bad_topos / sizeof *bad_topos; ++t) {
      setenv("FT_TOPO", bad_topos[t], 1);
      memset(out, 0, sizeof out);
      if (MPI_Allreduce_FT(in, out, 16, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD) != MPI_ERR_ARG) {
        printf("FT_TOPO=%s accepted on 1 rank\n", bad_topos[t]);
        ++bad;
      }
      bad += MPI_Allreduce_FT(MPI_IN_PLACE, out, 16, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD) != MPI_ERR_ARG;
    }
    setenv("FT_TOPO", "1", 1); /* the ring at any P: valid, the copy runs */
    memset(out, 0, sizeof out);
    bad += MPI_Allreduce_FT(in, out, 16, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD) != MPI_SUCCESS;
    bad += memcmp(in, out, 64) != 0;
    unsetenv("FT_TOPO");
    setenv("FT_LONELY", "1", 1); /* lonely ranks without FT_TOPO: invalid */
    bad += MPI_Allreduce_FT(in, out, 16, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD) != MPI_ERR_ARG;
    setenv("FT_LONELY", "0", 1); /* "0" is the same as unset */
    bad += MPI_Allreduce_FT(in, out, 16, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD) != MPI_SUCCESS;
    unsetenv("FT_LONELY");
    bad += MPI_Allreduce_FT(in, out, 16, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD) != MPI_SUCCESS;
  }
  MPI_Allreduce_FT_finalize();
  MPI_Finalize();
  printf(bad ? "mpi dtypes FAILED (%d)\n" : "mpi dtypes ok\n", bad);
  return bad != 0;
}
