#!/bin/bash
# fourth stream for B's look-ahead strip: A/B (debug 256 = strip before the trailing on B), factor tests
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_determinism.py tests/test_gpu_graph.py tests/test_gpu_parity.py tests/test_gpu_faults.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_four.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests_four.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/mask_ab.py 256 c3 c2 c5 > gpurun_out/four_ab.log 2>&1; echo "ab rc=$?"; grep -v amdgpu.ids gpurun_out/four_ab.log
