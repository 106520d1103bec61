# capture: probe case 11 (event re-recorded on another stream), then the group capture from C++ and pytest
mkdir -p gpurun_out
timeout -k 5 60 ./tools/capture/capture_probe 11 > gpurun_out/cap_probe11.log 2>&1; echo "case 11 rc=$?" >> gpurun_out/cap_probe11.log
for cfg in "2 1 10007 0" "2 2 64 0" "4 2,2 10007 4096" "8 8 100003 65536"; do
  timeout -k 5 60 ./tools/capture/group_capture $cfg >> gpurun_out/group_capture.log 2>&1; echo "[$cfg] rc=$?" >> gpurun_out/group_capture.log
done
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_allreduce.py -k "capture" -p no:cacheprovider > gpurun_out/pytest_capture.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_capture.log
cat gpurun_out/cap_probe11.log gpurun_out/group_capture.log; tail -12 gpurun_out/pytest_capture.log
