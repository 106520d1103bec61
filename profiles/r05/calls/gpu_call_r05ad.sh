#!/bin/bash
# Round 5, GPU call AD: which engine copies the host path's D2H pieces -- blit kernels or the copy engines --
# on plain streams and on high-priority streams (tools/ab_group/libftar_prio.so): kernel + copy traces of
# host_local (4 calls each).
cd "$(dirname "$0")/.." || exit 99
export TMPDIR=/tmp
O=gpurun_out/r05ad
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/plain -o hl -- \
  python3 -u -c "import json, bench; print(json.dumps(bench.host_local(steps=4)))" > $O/plain.log 2>&1 || exit 1
FTAR_LIB=$PWD/tools/ab_group/libftar_prio.so timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/prio -o hl -- \
  python3 -u -c "import json, bench; print(json.dumps(bench.host_local(steps=4)))" > $O/prio.log 2>&1 || exit 2
echo "call AD done"
