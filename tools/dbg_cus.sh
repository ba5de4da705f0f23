set -o pipefail
O=gpurun_out/${OUTD:-r05_s37}; mkdir -p $O
OUT=$O STEPS="tests" bash tools/gpu_round.sh || exit 1
for w in c2 c3; do timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-instrumented --no-batched --no-configs > $O/bench_$w.log 2>&1 || exit 1; done
for f in $O/bench_*; do echo $f; tail -1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('ms_per_step'), d['config']['blocking'])" ; done
