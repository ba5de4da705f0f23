set -o pipefail
O=gpurun_out/${OUTD:-r05_s34}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_panel_forms.py tests/test_gpu_faults.py tests/test_gpu_determinism.py tests/test_gpu_graph.py tests/test_gpu_mixed.py tests/test_gpu_headline.py -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1; tail -2 $O/t.log
timeout -k 10 100 ipm-zoo_amd/build/kbench_chain 11264 chainclk 512 > $O/chain11264.log 2>&1 || exit 1
timeout -k 10 60 ipm-zoo_amd/build/kbench_chain 2560 chainclk 512 > $O/chain2560.log 2>&1 || exit 1
grep -H "factor N" $O/*.log
for w in c3 c5 c2; do timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-instrumented --no-batched --no-configs > $O/bench_$w.log 2>&1 || exit 1; done
for f in $O/bench_*; do echo $f; tail -1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('ms_per_step'))" ; done
