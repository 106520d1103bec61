#!/bin/bash
# Round 5, GPU call AO: the in-process transport's copies-done event per message (FTAR_LOCAL_DONE=message)
# against one per receiving stream and flush (the default): engine_local three interleaved rounds and the
# group-call latency; the in-process GPU tests in message mode.
set -o pipefail
cd "$(dirname "$0")/.." || exit 99
export TMPDIR=/tmp
O=gpurun_out/r05ao
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 150 python3 -u bench.py --engine-local-only --steps 5 --warmup 2 > $O/el_stream_$i.json 2>> $O/el.err || exit 1
  FTAR_LOCAL_DONE=message timeout -k 10 150 python3 -u bench.py --engine-local-only --steps 5 --warmup 2 > $O/el_message_$i.json 2>> $O/el.err || exit 2
done
timeout -k 10 120 python3 -u tools/group_latency.py > $O/lat_stream.json 2>> $O/lat.err || exit 3
FTAR_LOCAL_DONE=message timeout -k 10 120 python3 -u tools/group_latency.py > $O/lat_message.json 2>> $O/lat.err || exit 4
FTAR_LOCAL_DONE=message timeout -k 10 600 python3 -u -m pytest tests/test_gpu_allreduce.py tests/test_gpu_peer.py -m gpu -q -x \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_message.log 2>&1 || exit 5
tail -1 $O/pytest_message.log
echo "call AO done"
