#!/bin/bash
# round 4, late: the whole GPU suite on the current tree, smoke(), and the N = 1 bench line
export TMPDIR=/tmp PYTHONUNBUFFERED=1; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; tail -c 600 gpurun_out/bench.log; exit $rc
