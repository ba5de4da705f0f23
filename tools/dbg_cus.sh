set -o pipefail
O=gpurun_out/${OUTD:-r05_s20}; mkdir -p $O
timeout -k 10 200 python bench.py --workload c4 --no-cpu-baseline > $O/bench_c4.log 2>&1 || exit 1
tail -1 $O/bench_c4.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phase_ms_per_step']); s=d.get('batched_shard',{}); print(s.get('value'), s.get('phase_ms_per_step'))"
OUT=$O STEPS="batchtests" bash tools/gpu_round.sh
