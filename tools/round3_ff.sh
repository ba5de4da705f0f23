#!/bin/bash
# C4 at one rank's share of the 8-GPU job (128 QPs) and at 1024, default flags
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --workload c4 --batch 128 --no-cpu-baseline > gpurun_out/ff_c4_128.log 2>&1; rc=$?; tail -c 600 gpurun_out/ff_c4_128.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline > gpurun_out/ff_c4_1024.log 2>&1; rc=$?; tail -c 600 gpurun_out/ff_c4_1024.log; exit $rc
