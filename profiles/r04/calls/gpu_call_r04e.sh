#!/bin/bash
# round 4: the peer-write trailing barrier -- the race test, the ASan RCCL stress that found it (progress lines
# keep the run from looking silent), and the peer / host-transport / exec-model / full-size suites
export TMPDIR=/tmp PYTHONUNBUFFERED=1; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_rccl_loopback.py -k copy_out > gpurun_out/write_race_after.log 2>&1; rc=$?; tail -3 gpurun_out/write_race_after.log; [ $rc -ne 0 ] && exit $rc
bash tools/asan/run.sh rccl 600 8 300 12 2 || exit $?
bash tools/asan/run.sh rccl 240 3 300 11 2 || exit $?
bash tools/asan/run.sh rccl 240 5 300 13 2 || exit $?
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_peer.py tests/test_gpu_host_transport.py tests/test_gpu_exec_model.py tests/test_gpu_full_size.py > gpurun_out/peer_suites.log 2>&1; rc=$?; tail -3 gpurun_out/peer_suites.log; exit $rc
