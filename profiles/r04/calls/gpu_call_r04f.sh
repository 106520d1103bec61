#!/bin/bash
# round 4: in-process group capture (serial on every runtime, per-rank forked streams refused), the capture
# depth probe, the engine stress (captures included) and the RCCL capture path
export TMPDIR=/tmp PYTHONUNBUFFERED=1; mkdir -p gpurun_out
timeout -k 10 300 bash tools/capture/depth_probe.sh > gpurun_out/capture_depth_probe.log 2>&1; cat gpurun_out/capture_depth_probe.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_allreduce.py -k "capture" tests/test_gpu_engine_stress.py tests/test_gpu_rccl_loopback.py::test_rccl_p2p_allreduce_captures_into_a_hip_graph > gpurun_out/capture_tests.log 2>&1; rc=$?; tail -5 gpurun_out/capture_tests.log; exit $rc
