# panel-path tests, chain clocks, then an A/B of this tree against _old: tools/run_st3.sh OUTDIR "WORKLOADS"
set -u
OUT=gpurun_out/$1; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_panel_forms.py tests/test_gpu_determinism.py tests/test_gpu_graph.py tests/test_gpu_headline.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
OUT=$OUT CHV="st" STEPS="chainclk_ab" bash tools/gpu_round.sh > /dev/null || exit 1
REPS="${REPS:-1 2}" bash tools/run_ab3.sh $1 "$2" . _old
