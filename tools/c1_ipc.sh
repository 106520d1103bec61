#!/bin/bash
# Buckets through ftar's MPI drop-in with 2 MPI ranks on the box's one GPU (the `ipc` transport: RCCL
# refuses ranks sharing a GPU): piece-pipelined host path (auto pieces, one piece) vs whole-bucket copies.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/c1_ipc
L=allreduce-over-mpi_amd/lib
run() {  # tag env... -- size
  local tag=$1; shift
  env FT_TOPO=1 FTAR_MPI_TRANSPORT=ipc "$@" timeout -k 10 120 /opt/conda/bin/mpiexec -n 2 \
    $L/ftar_benchmark --size $N --repeat 20 --warmup 3 --check > gpurun_out/c1_ipc/${tag}_$N.log 2>&1 || exit $?
  echo "$tag $(grep '^{' gpurun_out/c1_ipc/${tag}_$N.log)"
}
for N in ${SIZES:-1048576 16777216 67108864}; do
  run whole FTAR_HOST_PEER_PIPELINE=0
  run pipe FTAR_HOST_PEER_PIPELINE=1
  run pipe1piece FTAR_HOST_PEER_PIPELINE=1 FTAR_HOST_CHUNK_BYTES=1073741824
done
