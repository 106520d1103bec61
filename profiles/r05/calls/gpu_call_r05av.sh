#!/bin/bash
# Round 5, GPU call AV: the p2p host path with each D2H issued after the next step's work against right after
# its piece's last step (tools/ab_group/libftar_d2hnow.so): host_local, three interleaved rounds of 12 calls;
# then the host-buffer GPU tests.
cd "$(dirname "$0")/.." || exit 99
export TMPDIR=/tmp
O=gpurun_out/r05av
mkdir -p $O
hl() { timeout -k 10 120 python3 -u -c "import bench; d=bench.host_local(steps=12); print(d['ms_median'], d['ms_best'], sorted(d['ms_all'])[-1], d['check'][:12])" 2>/dev/null; }
for i in 1 2 3; do
  echo "deferred_$i $(hl)" || exit 1
  echo "now_$i $(FTAR_LIB=$PWD/tools/ab_group/libftar_d2hnow.so hl)" || exit 2
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_allreduce.py tests/test_gpu_full_size.py -m gpu -q -x -k host \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_host.log 2>&1 || { tail -3 $O/pytest_host.log; exit 3; }
tail -1 $O/pytest_host.log
echo "call AV done"
