#!/bin/bash
# One GPU-box session: smoke, GPU tests, bench, rocprof. Every GPU step has its
# own time limit; a fault/abort/timeout (exit >= 124) stops the script there.
# Usage: tools/gpu_run.sh [steps...]   steps: smoke tests testsall bench sweep prof pmc final ktree host hostipc hosttests dist1 dist2h dist4h dist2f peer2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
steps=("$@"); [ ${#steps[@]} -eq 0 ] && steps=(smoke tests bench prof)
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/summary.log
  local t0=$(date +%s)
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - t0 ))s)" | tee -a gpurun_out/summary.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc in $name: stopping"; exit $rc; fi
  return 0
}
for s in "${steps[@]}"; do
  case $s in
    smoke) run smoke 600 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run pytest_gpu 1200 python -m pytest tests -m gpu -q -x -p no:cacheprovider ;;
    testsall) run pytest_gpu 1200 python -m pytest tests -m gpu -q -p no:cacheprovider ;;
    bench) run bench 600 python bench.py --steps 20 --warmup 5 ;;
    sweep) run bench_sweep 600 python bench.py --steps 20 --warmup 5 --sweep --no-cpu-baseline ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
    # one tree, one box: the bench line, its kernel trace and both PMC passes, plus the tree's identity
    # (FTAR_COMMIT from the caller; the box has no .git) for tools/pmc_summary.py --meta
    final) python3 -c "import json, bench; json.dump({'commit': '${FTAR_COMMIT:-unknown}', 'kernel_sources_sha': bench.kernel_source_digest()}, open('gpurun_out/pmc_meta.json', 'w'))" &&
           run bench 600 python bench.py --steps 20 --warmup 5 &&
           run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline &&
           python3 tools/trace_split.py gpurun_out/prof/run_kernel_trace.csv --out gpurun_out/kernel_phases.json > /dev/null &&
           run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline &&
           run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline ;;
    pmc) run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline &&
         run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline ;;
    ktree) run kbench_tree 600 python tools/kbench.py --rounds 8 --dtypes f32,bf16 --shapes "8;2,4;4,2;2,2,2;4;2,2;16;4,4;2,2,2,2" ;;
    host) run hostpath 600 python tools/hostpath.py ;;
    hosttrace) run hosttrace 600 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/htrace -o run -- python3 tools/engine_trace.py --host --ranks 2 --topo 2 --elements 268435456 --host-chunk-bytes 4194304 --iters 2 ;;
    dist2h) FTAR_BENCH_BUDGET_S=150 run dist2h 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --host-comm --steps 5 --warmup 2 ;;
    dist4h) FTAR_BENCH_BUDGET_S=150 run dist4h 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29535 bench.py --host-comm --steps 5 --warmup 2 ;;
    dist2f) FTAR_BENCH_BUDGET_S=150 run dist2f 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29537 bench.py --steps 5 --warmup 2 ;;
    peer2) run peer2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29536 tools/peer_rehearsal.py ;;
    hostipc) run hostipc2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29538 tools/host_ipc_rate.py --sizes 24,26,28 --pieces 0,4194304 &&
             run hostipc4 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29539 tools/host_ipc_rate.py --sizes 24,26 --topo 4 ;;
    hosttests) run pytest_host 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_host_transport.py tests/test_harness.py -m gpu ;;
    hostcomm) run pytest_hostcomm 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider tests/test_gpu_full_size.py -k host_comm -m gpu ;;
    # the diagnostic gather's records on 2 ranks, and the IPC host pipeline's timing test
    glogtests) run pytest_glog 400 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_full_size.py::test_host_comm_gather_records tests/test_harness.py::test_harness_ipc_host_pipeline_beats_whole_bucket_copies -m gpu ;;
    # the ftar-free reproducer of DESIGN §6.4: 8 worker processes, copy streams at the highest priority, then plain
    xcdprobe) run xcdprobe 300 python3 -u tools/xcd_id_probe.py --procs 8 --iters ${XCD_ITERS:-400} --timeout 280 --out gpurun_out/xcd_probe.jsonl ${XCD_ARGS:-} &&
              run xcdprobe_plain 300 python3 -u tools/xcd_id_probe.py --procs 8 --iters ${XCD_ITERS:-400} --plain --timeout 280 --out gpurun_out/xcd_probe.jsonl ${XCD_ARGS:-} ;;
    # the same with the highest priority only, under the settings in XCD_ARGS (no plain control)
    xcdhi) run xcdhi 300 python3 -u tools/xcd_id_probe.py --procs 8 --iters ${XCD_ITERS:-400} --timeout 280 --out gpurun_out/xcd_probe.jsonl ${XCD_ARGS:-} ;;
    # stress_<config>[@cycles]: tools/host_comm_stress.py under one of its configurations
    stress_*) cfg=${s#stress_}; cyc=${cfg#*@}; [ "$cyc" = "$cfg" ] && cyc=${STRESS_CYCLES:-8}; cfg=${cfg%@*}
              run "stress_$cfg" 900 python -u tools/host_comm_stress.py --config "$cfg" --cycles "$cyc" --cases "${STRESS_CASES:-c4_read,c5_write,c4_host_read,c5_host_write}" --timeout 840 --world "${STRESS_WORLD:-8}" --out gpurun_out/stress.jsonl ;;
    # c4_host_read on 8 processes with the engine's hand-off marks, checked by tools/host_order_check.py --marks
    hbmarks) rm -f gpurun_out/marks.jsonl; FTAR_STRESS_MARKS=1 run hbmarks 600 python -u tools/host_comm_stress.py --config "${HB_CONFIG:-current}" --cycles "${STRESS_CYCLES:-4}" --cases c4_host_read --timeout 500 --out gpurun_out/marks.jsonl &&
             python3 tools/host_order_check.py --marks gpurun_out/marks.jsonl --out gpurun_out/marks_check.json ;;
    # one c4_host_read call on 8 processes, kernel + copy trace, for tools/host_order_check.py
    hbtrace) rm -f gpurun_out/pidmap.txt; FTAR_STRESS_PIDMAP=gpurun_out/pidmap.txt run hbtrace 600 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/hbtrace -- python3 tools/host_comm_stress.py --config "${HB_CONFIG:-current}" --cycles 1 --cases c4_host_read --timeout 500 ;;
    # engine_local under a kernel + copy trace, summarised per call (span, idle, fold time overlapped by transfers)
    eltrace) run eltrace 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/eltrace -o el -- python3 bench.py --engine-local-only --steps 5 --warmup 2 &&
             python3 tools/engine_local_trace.py gpurun_out/eltrace/el_kernel_trace.csv $(ls gpurun_out/eltrace/el_memory_copy_trace.csv 2>/dev/null) --first --calls 7 --keep 5 --hbm-bytes 39728447488 > gpurun_out/eltrace_summary.json ;;
    # the N > 1 line at P = 8 over RCCL loopback sockets on one GPU, at the driver's default budget (300 s)
    dist8lb) run dist8lb 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29561 bench.py --rccl-loopback --steps 3 --warmup 1 --elements 4194304 --elements-c5 4194304 --no-cpu-baseline --save-cost gpurun_out/node.cost &&
             grep '^{' gpurun_out/dist8lb.log > gpurun_out/dist8.json && python3 tools/scale_report.py gpurun_out/dist8.json > gpurun_out/dist8_report.txt ;;
    dist1) run dist1 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --force-dist --steps 5 --warmup 2 ;;
    *) echo "unknown step $s" ;;
  esac
done
