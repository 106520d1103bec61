#!/bin/bash
# Round 5, GPU call K: the in-process transport with one data-ready event per sending stream and one
# copies-done event per receiving stream per flush, and per-rank wake-ups, against the pooled-thread library
# before it (tools/ab_group/libftar_pool.so): group-call wall time and engine_local, alternating; then the
# default GPU suite on the new library.
set -o pipefail
cd "$(dirname "$0")/.." || exit 99
export TMPDIR=/tmp
O=gpurun_out/r05k
mkdir -p $O
OLD=$PWD/tools/ab_group/libftar_pool.so
for i in 1 2; do
  timeout -k 10 120 python3 -u tools/group_latency.py > $O/lat_new_$i.json 2>> $O/lat.err || exit 1
  FTAR_LIB=$OLD timeout -k 10 120 python3 -u tools/group_latency.py > $O/lat_old_$i.json 2>> $O/lat.err || exit 2
  timeout -k 10 120 python3 -u tools/group_latency.py --ranks 2 > $O/lat2_new_$i.json 2>> $O/lat.err || exit 3
  FTAR_LIB=$OLD timeout -k 10 120 python3 -u tools/group_latency.py --ranks 2 > $O/lat2_old_$i.json 2>> $O/lat.err || exit 4
done
for i in 1 2; do
  timeout -k 10 150 python3 -u bench.py --engine-local-only --steps 5 --warmup 2 > $O/el_new_$i.json 2>> $O/el.err || exit 5
  FTAR_LIB=$OLD timeout -k 10 150 python3 -u bench.py --engine-local-only --steps 5 --warmup 2 > $O/el_old_$i.json 2>> $O/el.err || exit 6
done
start=$(date +%s)
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --durations=20 \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || exit 7
echo "suite wall $(( $(date +%s) - start )) s" >> $O/pytest_gpu.log
echo "call K done"
