#!/bin/bash
# round 4, one GPU call: the execution-model engine tests and the RCCL bench rehearsal, the 8-rank RCCL
# loopback bench at C4's 1 GiB (enqueue times per form and piece), then the q16 ordering probe (last: it may
# end in a detected hang, which stops the script).  FINAL=1 first runs tools/gpu_run.sh final.
export TMPDIR=/tmp; mkdir -p gpurun_out
if [ -n "$FINAL" ]; then FTAR_COMMIT="${FTAR_COMMIT:-unknown}" bash tools/gpu_run.sh final || exit $?; fi
timeout -k 10 420 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_exec_model.py tests/test_gpu_peer.py "tests/test_gpu_bench_rehearsal.py::test_bench_n_gt_1_rehearsal_over_rccl" -m gpu > gpurun_out/pytest_exec_model.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_exec_model.log; [ $rc -ne 0 ] && exit $rc
FTAR_BENCH_BUDGET_S=480 FTAR_BENCH_SWEEP_S=330 timeout -k 10 540 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29571 bench.py --rccl-loopback --steps 3 --warmup 1 --no-cpu-baseline --no-host --no-c5 > gpurun_out/dist8_loopback_1GiB.json 2> gpurun_out/dist8_loopback_1GiB.err; rc=$?; tail -3 gpurun_out/dist8_loopback_1GiB.err; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
tools/rccl_order/run_probes.sh warm_opposite_q16
