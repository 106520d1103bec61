#!/bin/bash
# Round 5, GPU call B: the trimmed default GPU suite (its wall time is the check: < 450 s), then the
# engine_local pipeline at three fixed pieces next to the model's 64 MiB.
set -o pipefail
cd "$(dirname "$0")/.." || exit 99
export TMPDIR=/tmp
O=gpurun_out/r05b
mkdir -p $O
start=$(date +%s)
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --durations=60 \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || exit 1
echo "suite wall $(( $(date +%s) - start )) s" >> $O/pytest_gpu.log
for c in 16777216 33554432 134217728; do
  timeout -k 10 150 python3 -u bench.py --engine-local-only --steps 5 --warmup 2 --chunk-bytes $c \
    > $O/engine_local_piece_$c.json 2> $O/engine_local_piece.err || exit 2
done
echo "call B done"
