#!/bin/bash
# tools/asan/build/engine_stress on the GPU box (host sanitizers only; see engine_stress.cpp).
#   run.sh local SECONDS CALLS SEED          in-process groups
#   run.sh rccl SECONDS P CALLS SEED GENS    P processes over RCCL (loopback sockets)
#   run.sh host SECONDS P CALLS SEED GENS    P processes on the host-bootstrapped transport
cd "$(dirname "$0")" || exit 1
out=${GRAFT_REPO_ROOT:-../..}/gpurun_out/asan
mkdir -p "$out"
export ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0:halt_on_error=1:abort_on_error=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export HSA_ENABLE_IPC_MODE_LEGACY=0
mode=${1:-local}
if [ "$mode" = rccl ] || [ "$mode" = host ]; then
  log="$out/engine_stress_${mode}_p$3.log"
  timeout -k 10 "${2:-300}" ./build/engine_stress "$mode" "$3" "${4:-100}" "${5:-1}" "${6:-2}" > "$log" 2>&1
else
  log="$out/engine_stress.log"
  timeout -k 10 "${2:-600}" ./build/engine_stress "${3:-1500}" "${4:-1}" > "$log" 2>&1
fi
rc=$?
tail -5 "$log"
exit $rc
