cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_reduce.py -p no:cacheprovider > gpurun_out/pytest_reduce.log 2>&1 || { tail -20 gpurun_out/pytest_reduce.log; exit 1; }
tail -2 gpurun_out/pytest_reduce.log
bash tools/gpu_run.sh bench prof pmc
