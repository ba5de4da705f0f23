#!/bin/bash
# fourth stream (debug 256 = off) on torch's stream (as bench.py) and on the context's own stream
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
TORCH_STREAM=1 timeout -k 10 200 python -u tools/mask_ab.py 256 c3 c2 > gpurun_out/v_torch.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/v_torch.log | sed 's/^/torch /'; echo "rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/mask_ab.py 256 c3 c2 > gpurun_out/v_own.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/v_own.log | sed 's/^/own /'; echo "rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-batched > gpurun_out/v_bench.log 2>&1; rc=$?; echo "bench rc=$rc"; exit $rc
