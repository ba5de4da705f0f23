# C4 A/B: _old (HEAD worktree) vs this tree, bench c4 at B=1024 and 128, alternating; then the C4 tests
set -o pipefail
O=gpurun_out/${OUTD:-c4ab}; mkdir -p $O
for i in 1 2 3; do
  for w in old new; do
    d=.; [ $w = old ] && d=_old
    for b in 1024 128; do
      (cd $d && timeout -k 10 120 python bench.py --workload c4 --batch $b --no-cpu-baseline --steps 20) > $O/${w}_b${b}_$i.json 2>$O/${w}_b${b}_$i.err || exit 1
    done
  done
done
python - <<'PY' "$O"
import json,sys,glob,os
O=sys.argv[1]
for f in sorted(glob.glob(O+'/*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(os.path.basename(f), round(d['value']), {k:round(v,4) for k,v in d.get('phase_ms_per_step',{}).items()})
PY
timeout -k 10 500 python -u -m pytest tests/test_gpu_c4_batch.py tests/test_gpu_batch.py tests/test_gpu_graph.py tests/test_gpu_step_paths.py tests/test_gpu_determinism.py tests/test_gpu_formulations.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; tail -3 $O/tests.log
