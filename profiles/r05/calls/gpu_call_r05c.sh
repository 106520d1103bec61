#!/bin/bash
# Round 5, GPU call C: the engine_local trace on the committed transport (the runtime's copies), marker
# kernels between the calls, then the default GPU suite once more (its wall time: the < 450 s check).
set -o pipefail
cd "$(dirname "$0")/.." || exit 99
export TMPDIR=/tmp
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/el_trace -o el -- \
  python3 bench.py --engine-local-only --steps 5 --warmup 2 > $O/el_trace.log 2>&1 || exit 1
start=$(date +%s)
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --durations=40 \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || exit 2
echo "suite wall $(( $(date +%s) - start )) s" >> $O/pytest_gpu.log
echo "call C done"
