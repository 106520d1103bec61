#!/bin/bash
# tools/asan/build/engine_stress on the GPU box (host sanitizers only; see engine_stress.cpp)
cd "$(dirname "$0")" || exit 1
out=${GRAFT_REPO_ROOT:-../..}/gpurun_out/asan
mkdir -p "$out"
export ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0:halt_on_error=1:abort_on_error=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
timeout -k 10 "${1:-600}" ./build/engine_stress "${2:-1500}" "${3:-1}" > "$out/engine_stress.log" 2>&1
rc=$?
tail -5 "$out/engine_stress.log"
exit $rc
