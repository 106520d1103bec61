#!/bin/bash
# Round 5, GPU call Q: bench.py's host_local item (P = 2 in-process ranks, pinned 256 MiB host buckets) on the
# current library against the library before this round's late host-side changes (tools/ab_group/
# libftar_spawn.so), interleaved, 10 calls each.
set -o pipefail
cd "$(dirname "$0")/.." || exit 99
export TMPDIR=/tmp
O=gpurun_out/r05q
mkdir -p $O
OLD=$PWD/tools/ab_group/libftar_spawn.so
for i in 1 2 3; do
  timeout -k 10 120 python3 -u -c "import json, bench; print(json.dumps(bench.host_local(steps=10)))" > $O/hl_new_$i.json 2>> $O/hl.err || exit 1
  FTAR_LIB=$OLD timeout -k 10 120 python3 -u -c "import json, bench; print(json.dumps(bench.host_local(steps=10)))" > $O/hl_old_$i.json 2>> $O/hl.err || exit 2
done
echo "call Q done"
