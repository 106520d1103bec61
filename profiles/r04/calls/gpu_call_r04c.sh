#!/bin/bash
# round 4: the RCCL --comm-threads paths (refused on 4 queues, run with a queue each), the queue layout with
# lazily created host streams, then the whole GPU suite and smoke()
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_harness.py -k "refuses or queue_each or lifecycle" -m gpu > gpurun_out/pytest_harness_threads.log 2>&1; rc=$?; tail -8 gpurun_out/pytest_harness_threads.log; [ $rc -ne 0 ] && exit $rc
tools/rccl_order/run_probes.sh queues || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; exit $rc
