set -o pipefail
O=gpurun_out/${OUTD:-r05_s16}; mkdir -p $O
T="tests/test_gpu_graph.py -k mixed"

timeout -k 10 300 python -u -m pytest $T -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/t_early.log 2>&1; tail -3 $O/t_early.log

