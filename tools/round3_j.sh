#!/bin/bash
# merged look-ahead strip: kbench factor A/B (debug 128 = separate strip every period), GPU tests of the factor
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for N in 11264 16384 5632; do for d in 0 128; do
  KB_DEBUG=$d timeout -k 10 200 ipm-zoo_amd/build/kbench $N factor 512 > gpurun_out/kf_${N}_$d.log 2>&1; rc=$?; echo "N $N debug $d rc=$rc $(grep 'factor N' gpurun_out/kf_${N}_$d.log)"
  [ $rc -ne 0 ] && exit $rc
done; done
tail -3 /tmp/gr_i.out 2>/dev/null
timeout -k 10 200 ipm-zoo_amd/build/gemm_ref s > gpurun_out/gemmref32.log 2>&1; echo "gemmref rc=$?"; cat gpurun_out/gemmref32.log
