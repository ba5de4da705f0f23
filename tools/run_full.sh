# the whole -m gpu suite, then an A/B of this tree against _old on C2 / C3 / C5
set -u
OUT=gpurun_out/${RUNOUT:-r06_full}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
bash tools/run_ab3.sh ${RUNOUT:-r06_full} "${ABW:-c2 c3 c5}" . _old
