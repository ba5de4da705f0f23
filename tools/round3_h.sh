#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 ipm-zoo_amd/build/kbench_stamps 11264 factor 512 > gpurun_out/solve_stamps.log 2>&1; echo "stamps rc=$?"; grep solve gpurun_out/solve_stamps.log
