#!/bin/bash
# Round 5, GPU call AK: the 8-process host-comm full-size test (c4_host_read is the ipc host path, whose
# H2D and D2H now run on different queues at once) eight times on the current tree, and the ipc harness
# with --check at 2^26 eight times.  A failing test is a result; anything else ends the call.
cd "$(dirname "$0")/.." || exit 99
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05ak
mkdir -p $O
T=tests/test_gpu_full_size.py::test_host_comm_peer_forms_full_size_whole_bucket
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 300 python3 -u -m pytest $T -m gpu -q -x --timeout 280 --timeout-method thread -p no:cacheprovider > $O/t_$i.log 2>&1
  rc=$?
  echo "test $i rc=$rc $(grep -o 'c[45]_[a-z_]*: rank [0-9]*: [0-9]* elements differ[^\"]*' $O/t_$i.log | head -1)"
  [ $rc -le 1 ] || exit $rc
done
for i in 1 2 3 4 5 6 7 8; do
  FT_TOPO=1 FTAR_MPI_TRANSPORT=ipc timeout -k 10 120 /opt/conda/bin/mpiexec -n 2 allreduce-over-mpi_amd/lib/ftar_benchmark \
    --size 67108864 --repeat 10 --warmup 2 --check > $O/h_$i.log 2>&1 || exit 3
  echo "harness $i $(grep -c '(test passed)' $O/h_$i.log) passed, $(grep -o 'min time: [0-9.e-]*' $O/h_$i.log)"
done
echo "call AK done"
