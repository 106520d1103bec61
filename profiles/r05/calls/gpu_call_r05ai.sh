#!/bin/bash
# Round 5, GPU call AI: the ipc host path with its D2H pieces on the (idle) reduce stream, whose queue the
# H2D stream does not share (the copy streams shared one queue): the
# MPI drop-in (2 MPI ranks, ftar_benchmark --check) at 2^24 and 2^26, against the previous build
# (tools/ab_group/h_prev/), default queues, interleaved, and the new one with 8 queues; then the GPU tests of
# the host-bootstrapped communicator and the harness.
cd "$(dirname "$0")/.." || exit 99
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out/r05ai
mkdir -p $O
run() {  # tag dir N env...
  local tag=$1 dir=$2 N=$3; shift 3
  env FT_TOPO=1 FTAR_MPI_TRANSPORT=ipc "$@" timeout -k 10 120 /opt/conda/bin/mpiexec -n 2 \
    $dir/ftar_benchmark --size $N --repeat 20 --warmup 3 --check > $O/${tag}_$N.log 2>&1 || exit 1
  echo "$tag $N $(grep '^{' $O/${tag}_$N.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["min_s"]*1e3,3), round(d["avg_s"]*1e3,3), d["check"])')"
}
NEW=allreduce-over-mpi_amd/lib
OLD=tools/ab_group/h_prev
for i in 1 2; do
  for N in 16777216 67108864; do
    run new_$i $NEW $N
    run old_$i $OLD $N
  done
done
for N in 16777216 67108864; do run new_q8 $NEW $N GPU_MAX_HW_QUEUES=8; done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_full_size.py tests/test_gpu_host_transport.py tests/test_harness.py \
  -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -3 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
echo "call AI done"
