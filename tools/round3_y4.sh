#!/bin/bash
# the step on torch's default stream: which per-step caller-stream op costs (1024: no fork wait, 2048: no join wait)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in 1024 2048 3072; do
  TORCH_STREAM=1 timeout -k 10 200 python -u tools/mask_ab.py $m c3 > gpurun_out/y4_$m.log 2>&1; rc=$?
  grep "ms/step" gpurun_out/y4_$m.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
