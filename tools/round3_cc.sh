#!/bin/bash
# fp64 trailing update as the halving tree of rocBLAS DGEMM levels (debug 2048) vs the hand-written kernel
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/mask_ab.py 2048 c3 c3 > gpurun_out/cc_ab.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/cc_ab.log; exit $rc
