#!/bin/bash
# the fp32 conversion split over the chain and trailing streams: parity tests, then A/B (2048 = one launch)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_mixed.py tests/test_gpu_graph.py tests/test_gpu_step_paths.py tests/test_gpu_determinism.py tests/test_gpu_headline.py > gpurun_out/gg_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gg_tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/mask_ab.py 2048 c5 c5 > gpurun_out/gg_ab.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/gg_ab.log; exit $rc
