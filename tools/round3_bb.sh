#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_step_paths.py tests/test_gpu_graph.py > gpurun_out/bb_tests.log 2>&1; rc=$?; tail -15 gpurun_out/bb_tests.log; exit $rc
