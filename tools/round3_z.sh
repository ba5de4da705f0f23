#!/bin/bash
# kernel + HIP API traces of the C3 step on the context's own stream (0) and torch's default stream (1)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for ts in 0 1; do
  TORCH_STREAM=$ts timeout -k 10 240 rocprofv3 --kernel-trace --hip-trace --output-format csv -d gpurun_out/z_$ts -o run -- python3 tools/mask_ab.py 0 c3 > gpurun_out/z_$ts.log 2>&1; rc=$?
  grep "ms/step" gpurun_out/z_$ts.log | sed "s/^/ts=$ts /"; echo "ts=$ts rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
ls -la gpurun_out/z_0 gpurun_out/z_1
exit 0
