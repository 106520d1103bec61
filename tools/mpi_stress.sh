#!/bin/bash
# random calls through MPI_Allreduce_FT / _device (lib/ftar_mpi_stress), both transports; SAN=1: the
# host-sanitized build (tools/asan/build)
export NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 HSA_ENABLE_IPC_MODE_LEGACY=0
export ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0:halt_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
B=./allreduce-over-mpi_amd/lib/ftar_mpi_stress
[ "${SAN:-0}" = 1 ] && B=./tools/asan/build/ftar_mpi_stress
MPI=/opt/conda/bin/mpiexec
mkdir -p gpurun_out/mpi_stress
step() {  # name seconds env... -- command
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" env "$@" > gpurun_out/mpi_stress/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc: $(grep -c '"checked"' gpurun_out/mpi_stress/$name.log) ranks reported; $(grep -h '^FAIL' gpurun_out/mpi_stress/$name.log | head -2 | cut -c1-250)"
  [ $rc -ne 0 ] && ! { [ "${SAN:-0}" = 1 ] && grep -q "sanitizer_allocator_device.h:125" gpurun_out/mpi_stress/$name.log && [ "$(grep -c '"checked"' gpurun_out/mpi_stress/$name.log)" -gt 0 ] && ! grep -qE "ERROR: AddressSanitizer|runtime error|^FAIL" gpurun_out/mpi_stress/$name.log; } && exit $rc
  return 0
}
mpmd() {  # ranks args...: one NCCL_HOSTID per rank (RCCL between processes on one GPU)
  local n=$1; shift
  local cmd=()
  for ((r = 0; r < n; r++)); do
    [ $r -gt 0 ] && cmd+=(":")
    cmd+=(-n 1 -env NCCL_HOSTID "ftar-mpistress-$r" "$B" "$@")
  done
  printf '%s ' "${cmd[@]}"
}
step ipc2 170 FTAR_MPI_TRANSPORT=ipc $MPI -n 2 $B ${CALLS:-200} 401
step ipc4 170 FTAR_MPI_TRANSPORT=ipc $MPI -n 4 $B ${CALLS:-120} 402
step rccl2 170 FTAR_MPI_TRANSPORT=rccl $MPI $(mpmd 2 ${CALLS:-120} 403)
step rccl5 170 FTAR_MPI_TRANSPORT=rccl $MPI $(mpmd 5 ${CALLS:-60} 404)
