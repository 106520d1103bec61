#!/bin/bash
# Round 5, GPU call R: the bimodal host_local call time (17-20 ms or ~31 ms per call, either library):
# copy engines off (HSA_ENABLE_SDMA=0: blit kernels), and host pieces of 4 / 64 MiB against the default 16,
# interleaved with the default, 10 calls each.
set -o pipefail
cd "$(dirname "$0")/.." || exit 99
export TMPDIR=/tmp
O=gpurun_out/r05r
mkdir -p $O
run() { timeout -k 10 120 python3 -u -c "import json, bench; print(json.dumps(bench.host_local(steps=10)))"; }
for i in 1 2; do
  run > $O/hl_default_$i.json 2>> $O/hl.err || exit 1
  HSA_ENABLE_SDMA=0 run > $O/hl_nosdma_$i.json 2>> $O/hl.err || exit 2
  FTAR_HOST_CHUNK_BYTES=4194304 run > $O/hl_c4m_$i.json 2>> $O/hl.err || exit 3
  FTAR_HOST_CHUNK_BYTES=67108864 run > $O/hl_c64m_$i.json 2>> $O/hl.err || exit 4
done
echo "call R done"
