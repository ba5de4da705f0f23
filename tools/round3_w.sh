#!/bin/bash
# the r03_s4 build (tmp_old) vs HEAD on the same box, torch's stream and the context's own stream
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in old new old new; do
  for ts in 1 0; do
    if [ $v = old ]; then export IPMZ_PKG_DIR=$PWD/tmp_old/ipm-zoo_amd; else unset IPMZ_PKG_DIR; fi
    TORCH_STREAM=$ts timeout -k 10 200 python -u tools/mask_ab.py 0 c3 c2 > gpurun_out/w_$v$ts.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/w_$v$ts.log | sed "s/^/$v torch=$ts /"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
