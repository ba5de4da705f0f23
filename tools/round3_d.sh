#!/bin/bash
# solve per-block clocks (new M_J schedule), graph-capture probe (traced)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 ipm-zoo_amd/build/kbench_stamps 11264 factor 512 > gpurun_out/solve_stamps.log 2>&1; echo "stamps rc=$?"; grep -E "solve" gpurun_out/solve_stamps.log
PROBE_TRACE=1 timeout -k 10 120 python -u tools/dbg/graph_probe.py > gpurun_out/graph_trace.log 2>&1; echo "graph rc=$?"; grep -v "step: phase" gpurun_out/graph_trace.log | tail -60
