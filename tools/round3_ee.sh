#!/bin/bash
# eager factor join: only the chain stream A (debug 4096; A already waited for B, C, D) vs A, B, C (, D)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/mask_ab.py 4096 c3 c2 c5 > gpurun_out/ee_ab.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ee_ab.log
[ $rc -ne 0 ] && exit $rc
TORCH_STREAM=1 timeout -k 10 300 python -u tools/mask_ab.py 4096 c3 c2 > gpurun_out/ee_ab_torch.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ee_ab_torch.log | sed 's/^/torch /'; exit $rc
