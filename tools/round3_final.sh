#!/bin/bash
# round-3 validation: smoke, every GPU test, default bench line, kernel stats (profiles/r03_s5, r03_s6)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS="smoke tests bench prof" bash tools/gpu_round.sh || exit $?
