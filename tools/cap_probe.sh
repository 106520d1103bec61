# capture tests (shared-stream group capture + expected-failure shapes), and co-scheduling with 2 and 4 ranks
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_allreduce.py -k "capture or cu_mask" -p no:cacheprovider > gpurun_out/pytest_capture.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_capture.log
timeout -k 10 200 python tools/cosched.py --ranks 2 --elements 67108864 --cus 0,224,192,128 --chunks 16777216 > gpurun_out/cosched_p2.log 2>&1
timeout -k 10 200 python tools/cosched.py --ranks 4 --elements 67108864 --cus 0,224,192 --chunks 16777216 > gpurun_out/cosched_p4.log 2>&1
tail -8 gpurun_out/pytest_capture.log
