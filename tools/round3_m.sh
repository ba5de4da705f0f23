#!/bin/bash
# C4: first-touch KKT reads in the batched factor -- A/B, batch GPU tests
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_c4_batch.py tests/test_gpu_batch.py tests/test_gpu_formulations.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_c4.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests_c4.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -u tools/c4_ab.py > gpurun_out/c4_ab.log 2>&1; echo "ab rc=$?"; grep -v amdgpu.ids gpurun_out/c4_ab.log
