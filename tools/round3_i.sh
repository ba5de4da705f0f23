#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 ipm-zoo_amd/build/gemm_ref s > gpurun_out/gemmref32.log 2>&1; echo "rc=$?"; cat gpurun_out/gemmref32.log
