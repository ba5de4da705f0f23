#!/bin/bash
# the trivial-kernel fork/join pattern on torch's bundled HIP runtime (7.0)
export TMPDIR=/tmp
mkdir -p gpurun_out
for a in "mini 0" "mini 1" "mini 2" "mini 3" "mini 4" "mini 5" "mini 6" "mini 7"; do
  timeout -k 5 60 python -u tools/dbg/repro_torch.py $a > gpurun_out/repro.log 2>&1; rc=$?
  echo "args $a rc=$rc: $(grep -v 'amdgpu.ids' gpurun_out/repro.log | tr '\n' '|' | cut -c1-200)"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then exit $rc; fi
done
