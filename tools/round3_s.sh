#!/bin/bash
# C5 trailing update: SYRKX (W=0) vs the halving tree (W=512, 1024, 2048)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in 512 1024 2048 0 512 1024; do
  IPMZ_BLAS_W=$w timeout -k 10 200 python -u tools/blasw_check.py > gpurun_out/s_w$w.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/s_w$w.log; echo "W=$w rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
