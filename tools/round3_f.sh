#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/dbg/graph_probe.py > gpurun_out/graph_trace.log 2>&1; echo "graph rc=$?"; grep -v "step: phase" gpurun_out/graph_trace.log | tail -60
