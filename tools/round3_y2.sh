#!/bin/bash
# made on torch's stream / stepped on the own stream and the reverse
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "1 own" "0 torch" "1 -" "0 -"; do
  set -- $cfg
  ss=$2; [ "$ss" = "-" ] && ss=""
  TORCH_STREAM=$1 STEP_STREAM=$ss timeout -k 10 200 python -u tools/mask_ab.py 0 c3 > gpurun_out/y2_$1$2.log 2>&1; rc=$?
  grep "ms/step" gpurun_out/y2_$1$2.log | sed "s/^/made=$1 step=$2 /"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
