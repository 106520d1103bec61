#!/bin/bash
# Round 5, GPU call Z: the MPI drop-in's ipc host path (2 MPI ranks on the box's GPU, pieces pipelined)
# no longer beats whole-bucket copies (5.38 vs 5.20 ms at 2^24; round 2: 4.09).  Diagnostic: the same runs
# with 8 hardware queues per process (no queue shared by two engine streams).
cd "$(dirname "$0")/.." || exit 99
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05z
mkdir -p $O
L=allreduce-over-mpi_amd/lib
run() {  # tag N env...
  local tag=$1 N=$2; shift 2
  env FT_TOPO=1 FTAR_MPI_TRANSPORT=ipc "$@" timeout -k 10 120 /opt/conda/bin/mpiexec -n 2 \
    $L/ftar_benchmark --size $N --repeat 20 --warmup 3 --check > $O/${tag}_$N.log 2>&1 || exit 1
  echo "$tag $N $(grep '^{' $O/${tag}_$N.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["min_s"]*1e3, d["avg_s"]*1e3)')"
}
for N in 16777216 67108864; do
  run pipe_q4 $N FTAR_HOST_PEER_PIPELINE=1
  run pipe_q8 $N FTAR_HOST_PEER_PIPELINE=1 GPU_MAX_HW_QUEUES=8
  run whole_q4 $N FTAR_HOST_PEER_PIPELINE=0
  run pipe_q4b $N FTAR_HOST_PEER_PIPELINE=1
  run pipe_q8b $N FTAR_HOST_PEER_PIPELINE=1 GPU_MAX_HW_QUEUES=8
done
echo "call Z done"
