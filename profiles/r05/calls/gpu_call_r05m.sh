#!/bin/bash
# Round 5, GPU call M: the opt-in wide tests (FTAR_RUN_WIDE=1) after the group-call and in-process transport
# changes -- the in-process stress at 1,500 calls among them.
set -o pipefail
cd "$(dirname "$0")/.." || exit 99
export TMPDIR=/tmp
O=gpurun_out/r05m
mkdir -p $O
start=$(date +%s)
FTAR_RUN_WIDE=1 timeout -k 10 1000 python3 -u -m pytest tests -m "gpu and wide" -v --timeout 300 --timeout-method thread \
  --durations=20 -p no:cacheprovider > $O/pytest_wide.log 2>&1 || exit 1
echo "wide wall $(( $(date +%s) - start )) s" >> $O/pytest_wide.log
echo "call M done"
