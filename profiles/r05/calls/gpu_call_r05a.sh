#!/bin/bash
# Round 5, GPU call A: the engine on one GPU (bench.py's engine_local item, then its kernel + copy trace),
# the stream -> hardware-queue map with a CU-masked and the legacy NULL stream, the RCCL stress at the seed
# that stalled twice in round 4 (run once: the CU share is now refused on RCCL communicators), smoke, and
# the default N = 1 bench line.  Every GPU step has its own time limit; the first failure ends the call.
set -o pipefail
cd "$(dirname "$0")/.." || exit 99
export TMPDIR=/tmp
O=gpurun_out/r05a
mkdir -p $O
# A/B of the in-process transport's receive copies: the runtime's blit, one copy after another (round 4),
# against one launch of ftar's multi-segment copy per group (round 5); then the default once more
FTAR_LOCAL_COPY=runtime timeout -k 10 150 python3 -u bench.py --engine-local-only --steps 5 --warmup 2 > $O/engine_local_runtime.json 2> $O/engine_local_runtime.err || exit 1
timeout -k 10 150 python3 -u bench.py --engine-local-only --steps 5 --warmup 2 > $O/engine_local.json 2> $O/engine_local.err || exit 1
FTAR_LOCAL_COPY=runtime timeout -k 10 150 python3 -u bench.py --engine-local-only --steps 5 --warmup 2 > $O/engine_local_runtime2.json 2>> $O/engine_local_runtime.err || exit 1
timeout -k 10 150 python3 -u bench.py --engine-local-only --steps 5 --warmup 2 > $O/engine_local2.json 2>> $O/engine_local.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/el_trace -o el -- \
  python3 bench.py --engine-local-only --steps 5 --warmup 2 > $O/el_trace.log 2>&1 || exit 2
timeout -k 10 120 ./tools/rccl_order/queue_probe --masked --null > $O/queue_probe_masked_null.log 2>&1 || exit 3
FTAR_STRESS_VERBOSE=1 NCCL_IB_DISABLE=1 timeout -k 10 300 ./allreduce-over-mpi_amd/lib/ftar_engine_stress rccl 7 40 704 2 \
  > $O/stress_rccl7_seed704.log 2>&1 || exit 4
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 5
timeout -k 10 420 python3 -u bench.py > $O/bench.log 2>&1 || exit 6
echo "call A done"
