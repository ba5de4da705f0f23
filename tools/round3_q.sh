#!/bin/bash
# eager mixed-precision solve: host stop test (adaptive passes) vs all passes enqueued (debug 512)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mixed.py tests/test_gpu_graph.py tests/test_gpu_determinism.py tests/test_gpu_headline.py > gpurun_out/q_tests.log 2>&1; rc=$?; tail -3 gpurun_out/q_tests.log; echo "tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/mask_ab.py 512 c5 > gpurun_out/q_ab.log 2>&1; rc=$?; cat gpurun_out/q_ab.log; echo "ab rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 3 > gpurun_out/q_bench_c5.log 2>&1; rc=$?; tail -c 1500 gpurun_out/q_bench_c5.log; echo "bench rc=$rc"
exit $rc
