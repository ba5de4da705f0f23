set -o pipefail
O=gpurun_out/${OUTD:-r05_s32}; mkdir -p $O
for nbo in 512 256 384 512; do timeout -k 10 200 python bench.py --workload c2 --nbo $nbo --no-cpu-baseline --no-instrumented --no-batched --no-configs > $O/bench_c2_$nbo.log 2>&1 || exit 1; tail -1 $O/bench_c2_$nbo.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($nbo, d['value'], d.get('ms_per_step'))"; done
