#!/bin/bash
# the stress driver with per-call knobs (peer copy tuning, reduce CU share, RCCL registration, phase timing,
# alternating user streams): plain in-process and multi-process runs, and one sanitized in-process run
export NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 HSA_ENABLE_IPC_MODE_LEGACY=0
B=./allreduce-over-mpi_amd/lib/ftar_engine_stress
mkdir -p gpurun_out/soak
step() {  # name seconds args...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" $B "$@" > gpurun_out/soak/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc: $(grep -hE '^(rccl|host):|^\{"calls' gpurun_out/soak/$name.log | tail -1)"
  grep -h "^FAIL" gpurun_out/soak/$name.log | head -3 | cut -c1-300
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step knobs_local1 170 1400 301
step knobs_local2 170 1400 302
step knobs_rccl4 170 rccl 4 100 303 2
step knobs_host4 170 host 4 150 304 2
bash tools/asan/run.sh local 170 700 305 || exit $?
