#!/bin/bash
# round-3 session 2: validate HEAD (smoke, GPU tests, bench, kernel stats), solve/GEMM kernel benches, then the graph-capture probe (traced)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS="smoke tests bench prof" bash tools/gpu_round.sh || exit $?
timeout -k 10 200 ipm-zoo_amd/build/kbench 11264 factor 512 > gpurun_out/kfactor.log 2>&1; echo "kfactor rc=$?"; grep -E "factor N|solve" gpurun_out/kfactor.log
timeout -k 10 200 ipm-zoo_amd/build/kbench 16384 g32 0 1 2 3 4 5 6 7 > gpurun_out/g32.log 2>&1; echo "g32 rc=$?"; grep g32 gpurun_out/g32.log
PROBE_TRACE=1 timeout -k 10 120 python -u tools/dbg/graph_probe.py > gpurun_out/graph_trace.log 2>&1; echo "graph rc=$?"; grep -v "step: phase" gpurun_out/graph_trace.log | tail -40
