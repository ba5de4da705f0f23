set -u
OUT=gpurun_out/${RUNOUT:-r06_st}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_panel_forms.py tests/test_gpu_determinism.py tests/test_gpu_graph.py tests/test_gpu_headline.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
OUT=$OUT CHV="${CHVS:-st w0 st w0}" STEPS="chainclk_ab" bash tools/gpu_round.sh || exit 1
for i in 1 2; do
  TORCH_STREAM=1 timeout -k 10 200 python -u tools/mask_ab.py 0 c2 c3 > $OUT/ab_new_$i.log 2>&1 || exit 1
  TORCH_STREAM=1 IPMZ_PKG_DIR=_old/ipm-zoo_amd timeout -k 10 200 python -u tools/mask_ab.py 0 c2 c3 > $OUT/ab_old_$i.log 2>&1 || exit 1
done
grep -h "mask" $OUT/ab_*.log
