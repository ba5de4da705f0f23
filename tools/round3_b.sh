#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 ipm-zoo_amd/build/kbench 16384 g32 0 1 2 3 4 5 6 7 > gpurun_out/g32.log 2>&1; echo "g32 rc=$?"; cat gpurun_out/g32.log | grep g32
timeout -k 10 200 ipm-zoo_amd/build/kbench 11264 gvar 15 40 > gpurun_out/gvar.log 2>&1; echo "gvar rc=$?"; grep gvar gpurun_out/gvar.log
PROBE_TRACE=1 timeout -k 10 120 python -u tools/dbg/graph_probe.py > gpurun_out/graph_trace.log 2>&1; echo "graph rc=$?"; grep -v "step: phase" gpurun_out/graph_trace.log | tail -25
