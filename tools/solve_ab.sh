# persistent-solve change: per-hop clocks, the GPU tests, the bench line
set -o pipefail
O=gpurun_out/${OUTD:-solveab}; mkdir -p $O
for n in 11264 16384 2560; do timeout -k 10 100 ipm-zoo_amd/build/kbench_stamps $n solvecmp > $O/hops_$n.log 2>&1 || exit 1; done
grep -h "N=" $O/hops_*.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit 1
python - "$O/bench.log" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('c3', round(d['value'],2), d['phase_ms_per_step'])
for k,v in d['configs'].items(): print(k, round(v['value'],2), v['phase_ms_per_step'])
print('c4', round(d['batched']['value']), 'shard', round(d['batched_shard']['value']))
PY
