#!/bin/bash
# Round 5, GPU call AM: the order of call AB (where the one mismatch appeared, with high-priority streams):
# the ipc harness with --check at 2^24 and 2^26 four times each, then host_local twice, then the 8-process
# host-comm full-size test four times -- on the current tree (plain streams, D2H on the reduce stream).
cd "$(dirname "$0")/.." || exit 99
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05am
mkdir -p $O
for i in 1 2 3 4; do
  for N in 16777216 67108864; do
    FT_TOPO=1 FTAR_MPI_TRANSPORT=ipc timeout -k 10 120 /opt/conda/bin/mpiexec -n 2 allreduce-over-mpi_amd/lib/ftar_benchmark \
      --size $N --repeat 20 --warmup 3 --check > $O/h_${N}_$i.log 2>&1 || exit 1
    echo "harness $N $i $(grep -c '(test passed)' $O/h_${N}_$i.log) passed, $(grep -o 'min time: [0-9.e-]*' $O/h_${N}_$i.log)"
  done
done
for i in 1 2; do
  timeout -k 10 120 python3 -u -c "import bench; d=bench.host_local(steps=10); print('host_local', d['ms_median'], d['ms_best'], d['check'])" 2>/dev/null || exit 2
done
T=tests/test_gpu_full_size.py::test_host_comm_peer_forms_full_size_whole_bucket
for i in 1 2 3 4; do
  timeout -k 10 300 python3 -u -m pytest $T -m gpu -q -x --timeout 280 --timeout-method thread -p no:cacheprovider > $O/t_$i.log 2>&1
  rc=$?
  echo "test $i rc=$rc $(grep -o 'c[45]_[a-z_]*: rank [0-9]*: [0-9]* elements differ[^\"]*' $O/t_$i.log | head -1)"
  [ $rc -le 1 ] || exit $rc
done
echo "call AM done"
