#!/bin/bash
# Round 5, GPU call AC: test_host_comm_peer_forms_full_size_whole_bucket (8 processes, host-bootstrapped
# communicator, C4/C5 whole bucket) failed on c4_host_read with the host copy streams at high priority.
# Is the race ftar's, exposed by more concurrency, or the priority streams'?  The test on plain streams
# with 8 hardware queues per process (no queue shared), with the default 4, and the high-priority library
# once more.
cd "$(dirname "$0")/.." || exit 99
export TMPDIR=/tmp
O=gpurun_out/r05ac
mkdir -p $O
T=tests/test_gpu_full_size.py::test_host_comm_peer_forms_full_size_whole_bucket
pt() { timeout -k 10 300 python3 -u -m pytest $T -m gpu -q -x --timeout 280 --timeout-method thread -p no:cacheprovider; }
# a test that fails (rc 1) is a result; anything else (a time limit, an abort) ends the call
step() { local tag=$1; shift; env "$@" bash -c "$(declare -f pt); T=$T pt" > $O/$tag.log 2>&1; local rc=$?
         echo "$tag rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step plain_q8 GPU_MAX_HW_QUEUES=8
step plain_q4 GPU_MAX_HW_QUEUES=4
step prio_q4 FTAR_LIB=$PWD/tools/ab_group/libftar_prio.so GPU_MAX_HW_QUEUES=4
step prio_q8 FTAR_LIB=$PWD/tools/ab_group/libftar_prio.so GPU_MAX_HW_QUEUES=8
echo "call AC done"
