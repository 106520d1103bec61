#!/bin/bash
# ThreadSanitizer on the host code (tools/asan/Makefile with OUT=build_tsan SAN=-fsanitize=thread): in-process
# groups (one host thread per rank through the local hub) and the RCCL mode (the first-contact helper thread)
cd "$(dirname "$0")" || exit 1
out=${GRAFT_REPO_ROOT:-../..}/gpurun_out/asan
mkdir -p "$out"
export TSAN_OPTIONS="halt_on_error=0 report_signal_unsafe=0 history_size=2"
timeout -k 10 170 ./build_tsan/engine_stress 300 4 > "$out/tsan_local.log" 2>&1
echo "local rc=$?"; grep -c "WARNING: ThreadSanitizer" "$out/tsan_local.log"; tail -2 "$out/tsan_local.log"
timeout -k 10 170 ./build_tsan/engine_stress rccl 3 40 5 2 > "$out/tsan_rccl.log" 2>&1
echo "rccl rc=$?"; grep -c "WARNING: ThreadSanitizer" "$out/tsan_rccl.log"; tail -2 "$out/tsan_rccl.log"
exit 0
