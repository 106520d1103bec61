#!/bin/bash
# Round 5, GPU call W: host-mode H2D pieces issued two pieces ahead of the steps instead of all up front.
# host_local on the new library against the previous one (tools/ab_group/libftar_prev.so), interleaved, and
# the previous one with 8 hardware queues (no queue shared by two engine streams: the hypothesis); a trace of
# the new one; the host-buffer GPU tests.
set -o pipefail
cd "$(dirname "$0")/.." || exit 99
export TMPDIR=/tmp
O=gpurun_out/r05w
mkdir -p $O
PREV=$PWD/tools/ab_group/libftar_prev.so
run() { timeout -k 10 120 python3 -u -c "import json, bench; print(json.dumps(bench.host_local(steps=10)))"; }
for i in 1 2 3; do
  run > $O/hl_new_$i.json 2>> $O/hl.err || exit 1
  FTAR_LIB=$PREV run > $O/hl_prev_$i.json 2>> $O/hl.err || exit 2
done
FTAR_LIB=$PREV GPU_MAX_HW_QUEUES=8 run > $O/hl_prev_q8.json 2>> $O/hl.err || exit 3
GPU_MAX_HW_QUEUES=8 run > $O/hl_new_q8.json 2>> $O/hl.err || exit 4
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr -o hl -- \
  python3 -u -c "import json, bench; print(json.dumps(bench.host_local(steps=4)))" > $O/trace.log 2>&1 || exit 5
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_allreduce.py tests/test_gpu_full_size.py tests/test_gpu_host_transport.py \
  -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -k "host" > $O/pytest_host.log 2>&1 || exit 6
echo "call W done"
