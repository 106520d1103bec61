#!/bin/bash
# a longer sanitizer soak: more seeds, world sizes and calls than profiles/r04/calls/gpu_call_r04e.sh (each step stops the
# script on failure)
cd "$(dirname "$0")/../.." || exit 1
bash tools/asan/run.sh rccl 400 7 300 33 2 || exit $?
bash tools/asan/run.sh host 300 5 300 34 2 || exit $?
bash tools/asan/run.sh host 300 6 300 35 2 || exit $?
bash tools/asan/run.sh rccl 400 6 300 36 2 || exit $?
