export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_full_size.py tests/test_gpu_exec_model.py > gpurun_out/forms_full.log 2>&1
rc=$?; tail -3 gpurun_out/forms_full.log; exit $rc
