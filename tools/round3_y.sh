#!/bin/bash
# the step on torch's default stream (1), a torch side stream (2), the context's own stream (0)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for ts in 1 2 0 1 2 0; do
  TORCH_STREAM=$ts timeout -k 10 200 python -u tools/mask_ab.py 0 c3 c2 > gpurun_out/y_$ts.log 2>&1; rc=$?
  grep -v amdgpu.ids gpurun_out/y_$ts.log | sed "s/^/ts=$ts /"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
