#!/bin/bash
# Round 5, GPU call T: the in-process transport's batched receives (one multi-segment copy per stream and
# flush; the cross-device path) forced on every receive (FTAR_LOCAL_COPY=gather) through the in-process GPU
# tests, the stress tests on the default, and engine_local both ways.
set -o pipefail
cd "$(dirname "$0")/.." || exit 99
export TMPDIR=/tmp
O=gpurun_out/r05t
mkdir -p $O
FTAR_LOCAL_COPY=gather timeout -k 10 600 python3 -u -m pytest tests/test_gpu_allreduce.py tests/test_gpu_peer.py tests/test_gpu_exec_model.py \
  -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gather.log 2>&1 || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_engine_stress.py -m gpu -v -x --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_stress.log 2>&1 || exit 2
timeout -k 10 150 python3 -u bench.py --engine-local-only --steps 5 --warmup 2 > $O/el_default.json 2>> $O/el.err || exit 3
FTAR_LOCAL_COPY=gather timeout -k 10 150 python3 -u bench.py --engine-local-only --steps 5 --warmup 2 > $O/el_gather.json 2>> $O/el.err || exit 4
echo "call T done"
