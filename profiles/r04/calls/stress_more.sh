#!/bin/bash
# more seeds of the plain stress driver (captures, knobs, steered model)
export NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 HSA_ENABLE_IPC_MODE_LEGACY=0
B=./allreduce-over-mpi_amd/lib/ftar_engine_stress
mkdir -p gpurun_out/soak
step() {  # name seconds args...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" $B "$@" > gpurun_out/soak/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc: $(grep -hE '^(rccl|host):|^\{"calls' gpurun_out/soak/$name.log | tail -1)"
  grep -h "^FAIL" gpurun_out/soak/$name.log | head -2 | cut -c1-300
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step more_local1 170 1300 701
step more_local2 170 1300 702
step more_rccl6 170 rccl 6 40 703 2
step more_rccl7 170 rccl 7 30 704 2
step more_host5 170 host 5 80 705 2
