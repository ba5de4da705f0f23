#!/bin/bash
# wave-specialised persistent solve: A/B against the single-group kernel (kbench), per-block clocks, GPU tests
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for d in 0 128; do
  KB_DEBUG=$d timeout -k 10 200 ipm-zoo_amd/build/kbench 11264 factor 512 > gpurun_out/kfactor_$d.log 2>&1; rc=$?; echo "debug $d rc=$rc"; grep -E "solve" gpurun_out/kfactor_$d.log
  [ $rc -ne 0 ] && exit $rc
done
KB_DEBUG=0 timeout -k 10 200 ipm-zoo_amd/build/kbench 16384 factor 512 > gpurun_out/kfactor16k.log 2>&1; echo "16k rc=$?"; grep -E "solve" gpurun_out/kfactor16k.log
timeout -k 10 200 ipm-zoo_amd/build/kbench_stamps 11264 factor 512 > gpurun_out/solve_stamps.log 2>&1; echo "stamps rc=$?"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests.log 2>&1; echo "tests rc=$?"; tail -5 gpurun_out/tests.log
