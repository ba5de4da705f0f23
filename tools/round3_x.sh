#!/bin/bash
# hardware-queue sharing: GPU_MAX_HW_QUEUES 4 (default) vs 8, old (r03_s4) vs new build, torch's stream vs own
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for q in 8 4 8; do
  for v in new old; do
    for ts in 1 0; do
      if [ $v = old ]; then export IPMZ_PKG_DIR=$PWD/tmp_old/ipm-zoo_amd; else unset IPMZ_PKG_DIR; fi
      GPU_MAX_HW_QUEUES=$q TORCH_STREAM=$ts timeout -k 10 200 python -u tools/mask_ab.py 0 c3 c2 > gpurun_out/x_$q$v$ts.log 2>&1; rc=$?
      python3 - gpurun_out/x_$q$v$ts.log "q=$q $v torch=$ts" <<'PY'
import sys, re
t = {}
for l in open(sys.argv[1]):
    m = re.match(r"(c\d) mask \d+: ([\d.]+) ms", l)
    if m: t.setdefault(m.group(1), []).append(float(m.group(2)))
print(sys.argv[2], "  ".join(f"{k} {min(v):.3f}/{sorted(v)[len(v)//2]:.3f} ms" for k, v in t.items()))
PY
      [ $rc -ne 0 ] && exit $rc
    done
  done
done
exit 0
