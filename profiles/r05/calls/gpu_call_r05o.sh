#!/bin/bash
# Round 5, GPU call O: engine_local (8 in-process ranks, 16 engine streams on one GPU) with the process's
# hardware queues at HIP's default 4 against 8 and 16 (GPU_MAX_HW_QUEUES), interleaved; the group-call
# latency at 4 and 16.
set -o pipefail
cd "$(dirname "$0")/.." || exit 99
export TMPDIR=/tmp
O=gpurun_out/r05o
mkdir -p $O
for i in 1 2; do
  for q in 4 8 16; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 150 python3 -u bench.py --engine-local-only --steps 5 --warmup 2 > $O/el_q${q}_$i.json 2>> $O/el.err || exit 1
  done
done
for q in 4 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python3 -u tools/group_latency.py > $O/lat_q$q.json 2>> $O/lat.err || exit 2
done
echo "call O done"
