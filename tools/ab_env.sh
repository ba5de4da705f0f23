#!/bin/bash
# A/B a library env toggle on the bench: tools/ab_env.sh VAR "workloads" (alternating runs)
set -e
V=$1; WL=${2:-c3}
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for w in $WL; do
  for val in 0 1 0 1; do
    env $V=$val timeout -k 10 120 python bench.py --workload $w --no-cpu-baseline --steps 10 > gpurun_out/ab/${w}_$val.log 2>&1
    python3 -c "import json; d=json.loads(open('gpurun_out/ab/${w}_$val.log').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$V=$val $w', round(d['value'],2), {k: round(v,3) for k,v in d['phase_ms_per_step'].items()}, round(r.get('achieved',0),2))"
  done
done
