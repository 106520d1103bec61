#!/bin/bash
# Round 5, GPU call AB: the host path's copy streams at the highest priority (queues of their own) against
# plain streams (FTAR_HOST_STREAM_PRIO=0): the MPI drop-in's ipc host path (2 MPI ranks, ftar_benchmark) at
# 2^24 and 2^26, and host_local, interleaved; then the host-buffer GPU tests and the harness tests.
cd "$(dirname "$0")/.." || exit 99
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out/r05ab
mkdir -p $O
L=allreduce-over-mpi_amd/lib
run() {  # tag N env...
  local tag=$1 N=$2; shift 2
  env FT_TOPO=1 FTAR_MPI_TRANSPORT=ipc "$@" timeout -k 10 120 /opt/conda/bin/mpiexec -n 2 \
    $L/ftar_benchmark --size $N --repeat 20 --warmup 3 --check > $O/${tag}_$N.log 2>&1 || exit 1
  echo "$tag $N $(grep '^{' $O/${tag}_$N.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["min_s"]*1e3,3), round(d["avg_s"]*1e3,3), d["check"])')"
}
hl() { timeout -k 10 120 python3 -u -c "import json, bench; d=bench.host_local(steps=10); print(d['ms_median'], d['ms_best'], d['check'])"; }
for i in 1 2; do
  for N in 16777216 67108864; do
    run prio_$i $N
    run plain_$i $N FTAR_HOST_STREAM_PRIO=0
  done
  echo "host_local prio_$i $(hl)"
  echo "host_local plain_$i $(FTAR_HOST_STREAM_PRIO=0 hl)"
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_allreduce.py tests/test_gpu_full_size.py tests/test_gpu_host_transport.py tests/test_harness.py \
  -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -k "host or harness" > $O/pytest_host.log 2>&1 || exit 2
tail -1 $O/pytest_host.log
echo "call AB done"
