#!/bin/bash
# Round 5, GPU call F: the default GPU suite on the in-process transport's new receive copy, the engine_local
# trace of it, and the N = 1 bench line.
set -o pipefail
cd "$(dirname "$0")/.." || exit 99
export TMPDIR=/tmp
O=gpurun_out/r05f
mkdir -p $O
start=$(date +%s)
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --durations=20 \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || exit 1
echo "suite wall $(( $(date +%s) - start )) s" >> $O/pytest_gpu.log
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/el_trace -o el -- \
  python3 bench.py --engine-local-only --steps 5 --warmup 2 > $O/el_trace.log 2>&1 || exit 2
timeout -k 10 420 python3 -u bench.py > $O/bench.log 2>&1 || exit 3
echo "call F done"
