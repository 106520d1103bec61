#!/bin/bash
# The RCCL loopback soak over every data-movement form (peer forms and auto included), world sizes 2..8.
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
FTAR_RUN_WIDE=1 timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_rccl_loopback.py -k random_soak > gpurun_out/soak_forms.log 2>&1
rc=$?; tail -3 gpurun_out/soak_forms.log; exit $rc
