#!/bin/bash
# Round 5, GPU call E: A/B of the in-process transport's receive copy on one GPU (engine_local, interleaved):
# the runtime's blit per receive (default) against ftar's LDS-staged copy kernel per receive.
set -o pipefail
cd "$(dirname "$0")/.." || exit 99
export TMPDIR=/tmp
O=gpurun_out/r05e
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 150 python3 -u bench.py --engine-local-only --steps 7 --warmup 2 > $O/runtime_$i.json 2>> $O/err.log || exit 1
  FTAR_LOCAL_COPY=kernel timeout -k 10 150 python3 -u bench.py --engine-local-only --steps 7 --warmup 2 > $O/kernel_$i.json 2>> $O/err.log || exit 2
done
echo "call E done"
