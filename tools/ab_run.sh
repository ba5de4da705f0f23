#!/bin/bash
# A/B of a pytest selection: the tree at _old/ (a git worktree of an earlier
# commit, built in place) against this tree, then optional extra steps.
# Each GPU step under its own time limit; a crash / abort / timeout ends it.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
SEL=${SEL:-"tests/test_gpu_mixed.py"}
K=${K:-""}
run() {  # name timeout dir cmd...
  local name=$1 t=$2 dir=$3; shift 3
  echo "=== $name"
  (cd $dir && timeout -k 10 $t "$@") > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -4 $OUT/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name"; exit $rc; fi
}
for w in ${WHICH:-old new}; do
  d=.; [ $w = old ] && d=_old
  run ab_$w 400 $d python -u -m pytest $SEL ${K:+-k "$K"} -v --timeout 120 --timeout-method thread -p no:cacheprovider
done
for s in ${EXTRA:-}; do run $(basename $s .py) 240 . python -u $s; done
echo AB DONE
