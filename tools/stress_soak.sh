#!/bin/bash
# a soak of the plain stress driver (lib/ftar_engine_stress): more seeds than the GPU suite (the 8000-call
# in-process run is in profiles/r04/stress_soak/local_8k.log); RCCL over loopback sockets runs ~1 s per call at P = 8
export NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 HSA_ENABLE_IPC_MODE_LEGACY=0
B=./allreduce-over-mpi_amd/lib/ftar_engine_stress
mkdir -p gpurun_out/soak
step() {  # name seconds args...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" $B "$@" > gpurun_out/soak/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc: $(grep -hE '^(rccl|host):|^\{"calls' gpurun_out/soak/$name.log | tail -1)"
  grep -h "^FAIL" gpurun_out/soak/$name.log | head -3
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step rccl8 170 rccl 8 60 102 2
step rccl5 170 rccl 5 100 103 2
step host8 170 host 8 150 104 2
step rccl2 170 rccl 2 300 105 2
step host3 170 host 3 300 106 2
