#!/bin/bash
# Round 5, GPU call AJ: the default GPU suite after the ipc host path fixes (copy order, D2H on the reduce stream), the
# group-call latency (completion and enqueue), engine_local twice, smoke and the N = 1 bench line.
set -o pipefail
cd "$(dirname "$0")/.." || exit 99
export TMPDIR=/tmp
O=gpurun_out/r05aj
mkdir -p $O
start=$(date +%s)
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --durations=40 \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || exit 1
echo "suite wall $(( $(date +%s) - start )) s" >> $O/pytest_gpu.log
timeout -k 10 120 python3 -u tools/group_latency.py > $O/lat.json 2>> $O/lat.err || exit 2
timeout -k 10 120 python3 -u tools/group_latency.py --ranks 2 > $O/lat2.json 2>> $O/lat.err || exit 3
for i in 1 2; do
  timeout -k 10 150 python3 -u bench.py --engine-local-only --steps 5 --warmup 2 > $O/el_$i.json 2>> $O/el.err || exit 4
done
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 5
timeout -k 10 420 python3 -u bench.py > $O/bench.log 2>&1 || exit 6
echo "call AJ done"
