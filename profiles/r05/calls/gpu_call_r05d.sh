#!/bin/bash
# Round 5, GPU call D (one tree, one box): the default GPU suite, smoke, the N = 1 bench line, its kernel
# trace + stats, and both PMC passes (FETCH_SIZE, WRITE_SIZE in runs of their own) for tools/pmc_summary.py.
# Usage: tools/gpu_call_r05d.sh COMMIT
set -o pipefail
cd "$(dirname "$0")/.." || exit 99
export TMPDIR=/tmp
O=gpurun_out/r05d
mkdir -p $O
python3 -c "import json, bench; json.dump({'commit': '${1:-unknown}', 'kernel_sources_sha': bench.kernel_source_digest()}, open('$O/pmc_meta.json', 'w'))" || exit 98
start=$(date +%s)
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --durations=30 \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || exit 1
echo "suite wall $(( $(date +%s) - start )) s" >> $O/pytest_gpu.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 420 python3 -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit 3
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-engine-local > $O/prof.log 2>&1 || exit 4
python3 tools/trace_split.py $O/prof/run_kernel_trace.csv --out $O/kernel_phases.json > /dev/null || exit 5
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-engine-local > $O/pmc_fetch.log 2>&1 || exit 6
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-engine-local > $O/pmc_write.log 2>&1 || exit 7
echo "call D done"
