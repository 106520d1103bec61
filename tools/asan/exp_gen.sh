cd tools/asan
export ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0:halt_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p ../../gpurun_out/asan
timeout -k 10 300 ./build/engine_stress rccl 8 300 12 1 > ../../gpurun_out/asan/exp_gen1x300.log 2>&1; echo "gens=1 calls=300 rc=$?"
grep -E "^FAIL|^rccl:" ../../gpurun_out/asan/exp_gen1x300.log | cut -c1-300
FTAR_TRACE=1 timeout -k 10 300 ./build/engine_stress rccl 8 150 12 2 > ../../gpurun_out/asan/exp_trace.log 2>&1; echo "gens=2 trace rc=$?"
grep -E "^FAIL|^rccl:" ../../gpurun_out/asan/exp_trace.log | cut -c1-200
exit 0
