#!/bin/bash
# Round 5, GPU call S: host_local's piece per block (FTAR_HOST_CHUNK_BYTES) from 2 to 128 MiB (128 = whole
# blocks of the 256 MiB C3 bucket at P = 2), the order rotated per round, 10 calls each, three rounds.
set -o pipefail
cd "$(dirname "$0")/.." || exit 99
export TMPDIR=/tmp
O=gpurun_out/r05s
mkdir -p $O
run() { FTAR_HOST_CHUNK_BYTES=$1 timeout -k 10 120 python3 -u -c "import json, bench; print(json.dumps(bench.host_local(steps=10)))"; }
P="2 4 8 16 32 64 128"
for i in 1 2 3; do
  for m in $P; do
    run $((m << 20)) > $O/hl_c${m}m_$i.json 2>> $O/hl.err || exit 1
  done
  P="$(echo $P | awk '{for(i=2;i<=NF;i++) printf "%s ", $i; print $1}')"
done
echo "call S done"
