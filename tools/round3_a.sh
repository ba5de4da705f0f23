#!/bin/bash
# round-3 GPU batch: BK tests + timing, factor PMC passes (C3, C5, C4), kernel trace, graph-capture probe
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bk.py tests/test_gpu_eqnone.py -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/bk_tests.log 2>&1
rc=$?; echo "bk tests rc=$rc"; tail -3 gpurun_out/bk_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -u tools/bk_time.py 4096 11264 > gpurun_out/bk_time.log 2>&1 || exit $?
for w in c3 c5 c4; do PMCW=$w STEPS="pmcf_fetch pmcf_write pmcf_mops pmcf_busy" bash tools/gpu_round.sh > gpurun_out/pmc_$w.out 2>&1 || exit 1; done
echo pmc done
STEPS="trace graph" bash tools/gpu_round.sh
