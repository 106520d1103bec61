#!/bin/bash
# Round 5, GPU call H: the whole N > 1 bench line at P = 8 over RCCL itself (loopback sockets, one NCCL_HOSTID
# per rank, the ranks sharing the box's GPU; timings are not xGMI numbers): the round-5 fields end to end --
# form labels, c4_ring, the refit's unidentified constants and its saved calibration file, the C5 tie.
set -o pipefail
cd "$(dirname "$0")/.." || exit 99
export TMPDIR=/tmp
O=gpurun_out/r05h
mkdir -p $O
FTAR_BENCH_BUDGET_S=420 FTAR_BENCH_SWEEP_S=200 timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29561 bench.py --rccl-loopback --steps 3 --warmup 1 \
  --elements 4194304 --elements-c5 4194304 --no-cpu-baseline --save-cost $O/node.cost > $O/dist8.json 2> $O/dist8.err || exit 1
python3 tools/scale_report.py $O/dist8.json > $O/dist8_report.txt || exit 2
echo "call H done"
