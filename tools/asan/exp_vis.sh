cd tools/asan
export ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0:halt_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 HSA_ENABLE_IPC_MODE_LEGACY=0
o=../../gpurun_out/asan; mkdir -p $o
for v in "FTAR_DEBUG_COPYOUT_DMA=1" "FTAR_DEBUG_BARRIER_SYNC=1"; do
  env $v timeout -k 10 240 ./build/engine_stress rccl 8 300 12 1 > $o/exp_$v.log 2>&1; echo "$v rc=$?"
  grep -E "^FAIL|^rccl:" $o/exp_$v.log | cut -c1-250
done
exit 0
