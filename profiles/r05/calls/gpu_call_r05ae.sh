#!/bin/bash
# Round 5, GPU call AE: how often test_host_comm_peer_forms_full_size_whole_bucket mismatches with the host
# copy streams at high priority (one failure in three runs so far) against plain streams (the default):
# five runs each, alternating.  A failing test is a result; anything else ends the call.
cd "$(dirname "$0")/.." || exit 99
export TMPDIR=/tmp
O=gpurun_out/r05ae
mkdir -p $O
T=tests/test_gpu_full_size.py::test_host_comm_peer_forms_full_size_whole_bucket
for i in 1 2 3 4 5; do
  for v in plain prio; do
    if [ $v = prio ]; then export FTAR_LIB=$PWD/tools/ab_group/libftar_prio.so; else unset FTAR_LIB; fi
    timeout -k 10 300 python3 -u -m pytest $T -m gpu -q -x --timeout 280 --timeout-method thread -p no:cacheprovider > $O/${v}_$i.log 2>&1
    rc=$?
    echo "$v $i rc=$rc $(grep -o 'c[45]_[a-z_]*: rank [0-9]*: [0-9]* elements differ' $O/${v}_$i.log | head -1)"
    [ $rc -le 1 ] || exit $rc
  done
done
echo "call AE done"
