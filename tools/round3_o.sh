#!/bin/bash
# 16-byte write-through L^{-1} stores in the diagonal factor: kbench factor, new vs base build
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for N in 2560 11264; do for b in kbench kbench_base kbench kbench_base; do
  timeout -k 10 200 ipm-zoo_amd/build/$b $N factor 512 > gpurun_out/kf.log 2>&1; rc=$?; echo "$b N $N rc=$rc $(grep 'factor N' gpurun_out/kf.log)"
  [ $rc -ne 0 ] && exit $rc
done; done
