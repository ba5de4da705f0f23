#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 ipm-zoo_amd/build/gemm_ref x > gpurun_out/gemmref64x.log 2>&1; echo "rc=$?"; cat gpurun_out/gemmref64x.log
timeout -k 10 200 ipm-zoo_amd/build/kbench 11264 gvar 15 > gpurun_out/gvar15.log 2>&1; echo "rc=$?"; grep gvar gpurun_out/gvar15.log
