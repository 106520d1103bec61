#!/bin/bash
# in-process group captures on HIP 7.2 (/opt/rocm) with in-process groups always capturing serially
# (LocalTransport::capture_serially): every shape, on the capture stream ("shared") and on a stream forked per rank
B=./allreduce-over-mpi_amd/lib/ftar_capture_check
mkdir -p gpurun_out
run() {  # label env... -- args
  local label=$1; shift
  timeout -k 5 30 env "$@" > gpurun_out/capexp.log 2>&1; local rc=$?
  echo "$label rc=$rc: $(grep -E 'nodes|ok|differs' gpurun_out/capexp.log | tr '\n' ' ' | cut -c1-160)"
}
S="FTAR_REDUCE_SCATTER=stages FTAR_ALLGATHER=stages"
D="FTAR_REDUCE_SCATTER=direct FTAR_ALLGATHER=direct"
run "stages P3 t3 n2 shared"    $S $B 3 3 2 0 shared
run "direct P3 t1 n3000 shared" $D $B 3 1 3000 0 shared
run "direct P8 t8 n100003 shared" $D $B 8 8 100003 0 shared
run "stages P8 t1 n100003 c4096 shared" $S $B 8 1 100003 4096 shared
run "direct P2 t1 n3000 c4096 forked-per-rank" $D $B 2 1 3000 4096
run "direct P3 t1 n3000 forked-per-rank" $D $B 3 1 3000 0
run "direct P4 t2,2 n3000 forked-per-rank" $D $B 4 2,2 3000 0
run "direct P8 t8 n100003 forked-per-rank" $D $B 8 8 100003 0
run "stages P5 t2,2+1 n1003 c4096 forked-per-rank" $S $B 5 2,2 1003 4096 forked 1
exit 0
