#!/bin/bash
# CU reservation for the chain / rows streams (IPMZ_CU_RESERVE=r) vs shared CUs
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 0 32 16 64 0 32; do
  IPMZ_CU_RESERVE=$r timeout -k 10 200 python -u tools/mask_ab.py 0 c3 c2 > gpurun_out/t_r$r.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/t_r$r.log | sed "s/^/r=$r /"; echo "r=$r rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
