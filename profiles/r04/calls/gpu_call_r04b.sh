#!/bin/bash
# round 4: the peer-form teardown abort of test_gpu_exec_model (steer2), uncaptured (-s) so the runtime's own
# message is kept; stops at the first failure
export TMPDIR=/tmp; mkdir -p gpurun_out
AMD_LOG_LEVEL=1 timeout -k 10 300 python -u -m pytest -s -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_exec_model.py -k "steer2 and 4-4" -m gpu > gpurun_out/pytest_exec_model_diag.log 2>&1; rc=$?; tail -30 gpurun_out/pytest_exec_model_diag.log; exit $rc
