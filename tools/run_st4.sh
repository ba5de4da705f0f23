# panel-path tests, one serialized-dispatch (rocprofv3 --pmc) C2 and C3 pass, then an A/B against _old
set -u
OUT=gpurun_out/$1; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_panel_forms.py tests/test_gpu_determinism.py tests/test_gpu_graph.py tests/test_gpu_headline.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
for w in c2 c3; do PMCW=$w OUT=$OUT STEPS="pmcf_fetch" bash tools/gpu_round.sh > /dev/null || exit 1; grep -c "timed out" $OUT/${w}_pmcf_fetch.log; tail -2 $OUT/${w}_pmcf_fetch.log | head -1; done
REPS="${REPS:-1 2}" bash tools/run_ab3.sh $1 "$2" . _old
