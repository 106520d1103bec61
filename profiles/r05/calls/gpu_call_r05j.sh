#!/bin/bash
# Round 5, GPU call J: the group calls' pooled rank threads against one std::thread per rank per call (the
# previous library, tools/ab_group/libftar_spawn.so): group-call wall time at small to large buckets and
# the engine_local item, alternating; then the GPU tests of the in-process group calls on the pool.
set -o pipefail
cd "$(dirname "$0")/.." || exit 99
export TMPDIR=/tmp
O=gpurun_out/r05j
mkdir -p $O
SPAWN=$PWD/tools/ab_group/libftar_spawn.so
for i in 1 2; do
  timeout -k 10 120 python3 -u tools/group_latency.py > $O/lat_pool_$i.json 2>> $O/lat.err || exit 1
  FTAR_LIB=$SPAWN timeout -k 10 120 python3 -u tools/group_latency.py > $O/lat_spawn_$i.json 2>> $O/lat.err || exit 2
  timeout -k 10 120 python3 -u tools/group_latency.py --ranks 2 > $O/lat2_pool_$i.json 2>> $O/lat.err || exit 3
  FTAR_LIB=$SPAWN timeout -k 10 120 python3 -u tools/group_latency.py --ranks 2 > $O/lat2_spawn_$i.json 2>> $O/lat.err || exit 4
done
for i in 1 2; do
  timeout -k 10 150 python3 -u bench.py --engine-local-only --steps 5 --warmup 2 > $O/el_pool_$i.json 2>> $O/el.err || exit 5
  FTAR_LIB=$SPAWN timeout -k 10 150 python3 -u bench.py --engine-local-only --steps 5 --warmup 2 > $O/el_spawn_$i.json 2>> $O/el.err || exit 6
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_allreduce.py tests/test_gpu_engine_stress.py tests/test_gpu_peer.py \
  -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_group.log 2>&1 || exit 7
echo "call J done"
