#!/bin/bash
# Host-path / harness / reference-CPU measurements on the GPU box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=allreduce-over-mpi_amd/lib
nproc > gpurun_out/host_nproc.txt; lscpu > gpurun_out/lscpu.txt 2>&1
# C1: the reference's own CPU/MPI path (P=2 ring, 2^20 fp32), benchmark.cpp timing
FT_TOPO=1 timeout -k 10 120 /opt/conda/bin/mpiexec -n 2 oracle/_ref/ref_golden arbench --n 1048576 --repeat 50 > gpurun_out/ref_c1.json 2>gpurun_out/ref_c1.err
FT_TOPO=2 timeout -k 10 120 /opt/conda/bin/mpiexec -n 2 oracle/_ref/ref_golden arbench --n 1048576 --repeat 50 > gpurun_out/ref_c1_tree.json 2>>gpurun_out/ref_c1.err
FT_TOPO=1 timeout -k 10 300 /opt/conda/bin/mpiexec -n 8 oracle/_ref/ref_golden arbench --n 16777216 --repeat 10 > gpurun_out/ref_p8_ring.json 2>>gpurun_out/ref_c1.err
FT_TOPO=1 timeout -k 10 120 /opt/conda/bin/mpiexec -n 2 $L/ftar_benchmark --comm-type mpi --size 1048576 --repeat 50 > gpurun_out/mpich_c1.log 2>&1
# the product harness, one rank (host buffers and device-resident)
timeout -k 10 300 /opt/conda/bin/mpiexec -n 1 $L/ftar_benchmark --size 67108864 --repeat 10 --warmup 2 --check > gpurun_out/ftarbench_host.log 2>&1 &&
timeout -k 10 300 /opt/conda/bin/mpiexec -n 1 $L/ftar_benchmark --size 67108864 --repeat 10 --warmup 2 --check --device > gpurun_out/ftarbench_dev.log 2>&1 &&
timeout -k 10 600 python tools/hostpath.py > gpurun_out/hostpath.log 2>&1
echo "rc=$?"
tail -3 gpurun_out/ref_c1.json gpurun_out/ref_c1_tree.json gpurun_out/ref_p8_ring.json gpurun_out/mpich_c1.log gpurun_out/ftarbench_host.log gpurun_out/ftarbench_dev.log gpurun_out/hostpath.log
