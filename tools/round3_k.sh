#!/bin/bash
# rocBLAS SYRKX fp32 trailing update: C5 A/B in the bench process, mixed-precision GPU tests
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/blas_ab.py > gpurun_out/blas_ab.log 2>&1; rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/blas_ab.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_mixed.py tests/test_gpu_headline.py tests/test_gpu_determinism.py tests/test_gpu_graph.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_mixed.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/tests_mixed.log
