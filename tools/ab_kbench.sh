#!/bin/bash
# A/B of the factor: kbench (factor + solve) and bench legs in _old (baseline worktree) and this tree
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in old new; do
  d=.; [ $w = old ] && d=_old
  for N in ${KN:-2560 11264}; do
    (cd $d && timeout -k 10 120 ipm-zoo_amd/build/kbench $N factor ${KNBO:-512}) > gpurun_out/kb_${w}_$N.log 2>&1 || { echo "kbench $w $N failed"; exit 1; }
    grep -E "factor N|persistent solve" gpurun_out/kb_${w}_$N.log | sed "s/^/$w: /"
  done
done
for w in ${BENCH:-}; do
  for rep in old new; do
    d=.; [ $rep = old ] && d=_old
    (cd $d && timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-batched --no-configs) > gpurun_out/bench_${rep}_$w.log 2>&1 || { echo "bench $rep $w failed"; exit 1; }
    python -c "import json,sys;d=json.loads(open('gpurun_out/bench_${rep}_$w.log').read().strip().splitlines()[-1]);print('$rep $w', round(d['value'],2), d['phase_ms_per_step'])"
  done
done
echo AB DONE
