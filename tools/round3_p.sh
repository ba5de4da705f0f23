#!/bin/bash
# one-workgroup batched factor: 8 waves (one QP per CU at a time) vs 4 waves (two QPs per CU), kbench small
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for d in 0 512 0 512; do
  KB_DEBUG=$d timeout -k 10 200 ipm-zoo_amd/build/kbench 320 small > gpurun_out/small_$d.log 2>&1; rc=$?; echo "debug $d rc=$rc $(grep 'small factor' gpurun_out/small_$d.log | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
done
