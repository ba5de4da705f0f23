#!/bin/bash
# capture fix: minimal patterns with noted dependencies, the product probe (eager vs graph directions), graph vs eager timing
export TMPDIR=/tmp
mkdir -p gpurun_out
for a in "mini 10" "mini 11"; do
  timeout -k 5 60 python -u tools/dbg/repro_torch.py $a > gpurun_out/repro.log 2>&1; rc=$?
  echo "args $a rc=$rc: $(grep -v 'amdgpu.ids' gpurun_out/repro.log | tr '\n' '|' | cut -c1-300)"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then exit $rc; fi
done
timeout -k 10 120 python -u tools/dbg/graph_probe.py 1024,256,128 2048,512,0 > gpurun_out/graph_probe.log 2>&1; rc=$?; echo "probe rc=$rc"; grep -v "amdgpu.ids\|2d34a8" gpurun_out/graph_probe.log | tail -24
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/graph_ab.py c2 c3 c5 > gpurun_out/graph_ab.log 2>&1; echo "ab rc=$?"; cat gpurun_out/graph_ab.log | grep -v amdgpu.ids
