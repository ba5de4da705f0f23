#!/bin/bash
# kernel traces of the current C5 and C4 steps (factor timeline / phase analysis)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r_c5 -o c5 -- python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --no-batched --no-instrumented > gpurun_out/r_c5.log 2>&1; rc=$?; echo "c5 rc=$rc"; tail -c 400 gpurun_out/r_c5.log
[ $rc -ne 0 ] && exit $rc
find gpurun_out/r_c5 -name "*kernel_trace.csv" | head -3
exit 0
