set -o pipefail
O=gpurun_out/${OUTD:-r05_pmc2}; mkdir -p $O
PMCW=c2 OUT=$O STEPS="pmcf_fetch pmcf_write pmcf_mops pmcf_busy" bash tools/gpu_round.sh || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_panel_forms.py tests/test_gpu_faults.py tests/test_gpu_graph.py -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1; tail -2 $O/t.log
timeout -k 10 60 ipm-zoo_amd/build/kbench_chain 2560 chainclk 512 > $O/chain2560.log 2>&1 || exit 1
head -4 $O/chain2560.log
timeout -k 10 200 python bench.py --workload c2 --no-cpu-baseline --no-instrumented --no-batched --no-configs > $O/bench_c2.log 2>&1 || exit 1
tail -1 $O/bench_c2.log | cut -c1-200
