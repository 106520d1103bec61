#!/bin/bash
# Round 5, GPU call X: host_local with the H2D lookahead at 0, 1, 2 (in-tree), 4 pieces and the previous
# all-up-front library, the order rotated per round, 10 calls each, three rounds.
set -o pipefail
cd "$(dirname "$0")/.." || exit 99
export TMPDIR=/tmp
O=gpurun_out/r05x
mkdir -p $O
A=$PWD/tools/ab_group
run() { timeout -k 10 120 python3 -u -c "import json, bench; print(json.dumps(bench.host_local(steps=10)))"; }
V="la0 la1 la2 la4 prev"
for i in 1 2 3; do
  for v in $V; do
    if [ "$v" = la2 ]; then run > $O/hl_${v}_$i.json 2>> $O/hl.err || exit 1
    else FTAR_LIB=$A/libftar_$v.so run > $O/hl_${v}_$i.json 2>> $O/hl.err || exit 2; fi
  done
  V="$(echo $V | awk '{for(i=2;i<=NF;i++) printf "%s ", $i; print $1}')"
done
echo "call X done"
