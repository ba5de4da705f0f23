#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/c4_split_ab.py > gpurun_out/u_split.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/u_split.log; echo "rc=$rc"; exit $rc
