#!/bin/bash
# C5: the smallest trailing order that takes the rocBLAS path (experiment build, XP_MIN_R)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 4096 2048 1024 4096 2048 1024; do
  XP_MIN_R=$r timeout -k 10 200 python -u tools/mask_ab.py 0 c5 > gpurun_out/dd_$r.log 2>&1; rc=$?
  grep "ms/step" gpurun_out/dd_$r.log | sed "s/^/min_r=$r /"; [ $rc -ne 0 ] && exit $rc
done
exit 0
