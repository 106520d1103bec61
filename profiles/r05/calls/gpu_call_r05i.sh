#!/bin/bash
# Round 5, GPU call I: the default GPU suite after the MPI drop-in's calibration-file check, smoke
# and the N = 1 bench line.
set -o pipefail
cd "$(dirname "$0")/.." || exit 99
export TMPDIR=/tmp
O=gpurun_out/r05i
mkdir -p $O
start=$(date +%s)
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --durations=20 \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || exit 1
echo "suite wall $(( $(date +%s) - start )) s" >> $O/pytest_gpu.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 420 python3 -u bench.py > $O/bench.log 2>&1 || exit 3
echo "call I done"
