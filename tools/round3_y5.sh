#!/bin/bash
# the forked step on torch's default stream (1), a torch side stream (2), the own stream (0): host-joined
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for ts in 1 2 0 1; do
  TORCH_STREAM=$ts timeout -k 10 200 python -u tools/mask_ab.py 0 c3 c2 c5 > gpurun_out/y5_$ts.log 2>&1; rc=$?
  grep "ms/step" gpurun_out/y5_$ts.log | sed "s/^/ts=$ts /"
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/y5_bench.log 2>&1; rc=$?; echo "bench rc=$rc"
exit $rc
