#!/bin/bash
# C5 factor-phase counter passes with the rocBLAS halving-tree trailing update (profiles/factor_traffic_c5.json)
set -u
export TMPDIR=/tmp
PMCW=c5 STEPS="pmcf_fetch pmcf_write pmcf_mops pmcf_busy" bash tools/gpu_round.sh
