#!/bin/bash
# fourth look-ahead stream on (0) vs not forked at all (256), own stream, and the r03_s4 build
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in new old new; do
  if [ $v = old ]; then export IPMZ_PKG_DIR=$PWD/tmp_old/ipm-zoo_amd; else unset IPMZ_PKG_DIR; fi
  timeout -k 10 300 python -u tools/mask_ab.py 256 c3 c2 c5 > gpurun_out/aa_$v.log 2>&1; rc=$?
  grep "ms/step" gpurun_out/aa_$v.log | sed "s/^/$v /"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
