#!/bin/bash
# One GPU-box session: smoke -> GPU tests -> bench -> rocprof kernel stats.
# Every GPU step has its own time limit; a crash/abort/timeout ends the run
# (exit codes 124/134/137/139 or negative), plain test failures (1) do not.
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$(basename "$1") t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in ${STEPS:-smoke tests bench prof}; do
  case $s in
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) step tests 1000 python -u -m pytest tests -m gpu -v --timeout=400 --timeout-method thread -p no:cacheprovider ;;
    bench) step bench 600 python bench.py ${BENCH_ARGS:-} ;;
    bench_c2) step bench_c2 300 python bench.py --workload c2 ;;
    bench_c4) step bench_c4 300 python bench.py --workload c4 ;;
    bench_c5) step bench_c5 300 python bench.py --workload c5 ;;
    prof)  step prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline ;;
    # HBM traffic: one counter group per pass (MI355X_MICROARCH.md, rocprofv3 PMC slots)
    pmc_fetch) step pmc_fetch 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline ;;
    pmc_write) step pmc_write 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline ;;
    # factor-phase counters of ONE bench step (tools/pmc_factor.py), one counter group per pass
    pmcf_fetch) step ${PMCW:-c3}_pmcf_fetch 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/${PMCW:-c3}_pmcf_fetch" -o run --output-format csv -- python bench.py --workload ${PMCW:-c3} --steps 1 --warmup 0 --no-cpu-baseline --no-instrumented --no-batched --no-configs ;;
    pmcf_write) step ${PMCW:-c3}_pmcf_write 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/${PMCW:-c3}_pmcf_write" -o run --output-format csv -- python bench.py --workload ${PMCW:-c3} --steps 1 --warmup 0 --no-cpu-baseline --no-instrumented --no-batched --no-configs ;;
    # (two small passes: one 4-counter pass slows every dispatch enough that the
    # panel path's cross-launch hand-offs can time out under the profiler)
    pmcf_mops) step ${PMCW:-c3}_pmcf_mops 240 rocprofv3 --pmc $([ "${PMCW:-c3}" = c5 ] && echo SQ_INSTS_VALU_MFMA_MOPS_F32 || echo SQ_INSTS_VALU_MFMA_MOPS_F64) -d "$OUT/${PMCW:-c3}_pmcf_mops" -o run --output-format csv -- python bench.py --workload ${PMCW:-c3} --steps 1 --warmup 0 --no-cpu-baseline --no-instrumented --no-batched --no-configs ;;
    pmcf_busy) step ${PMCW:-c3}_pmcf_busy 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES -d "$OUT/${PMCW:-c3}_pmcf_busy" -o run --output-format csv -- python bench.py --workload ${PMCW:-c3} --steps 1 --warmup 0 --no-cpu-baseline --no-instrumented --no-batched --no-configs ;;
    # (kbench / sgemm_bench are listed in .gpurunignore: drop those lines to run the experiment steps)
    kbench) step kbench 300 ipm-zoo_amd/build/kbench 11264 ;;
    sgemm) step sgemm 200 ipm-zoo_amd/build/sgemm_bench ${SGEMM_R:-15872} ${SGEMM_V:-} ;;
    smallv) step smallv 100 ipm-zoo_amd/build/kbench 320 smallv ;;
    ab64) TORCH_STREAM=1 step ab64 300 python -u tools/mask_ab.py 1024 c3 ;;
    ab32) TORCH_STREAM=1 step ab32 300 python -u tools/mask_ab.py 128 c5 ;;
    c4ab) step c4ab 300 python -u tools/c4_ab.py 8192 ;;
    batchtests) step batchtests 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_c4_batch.py tests/test_gpu_formulations.py tests/test_gpu_dist.py -v --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    c2old) TORCH_STREAM=1 IPMZ_PKG_DIR=_old/ipm-zoo_amd step c2old 200 python -u tools/mask_ab.py 0 c2 c3 ;;
    c2new) TORCH_STREAM=1 step c2new 200 python -u tools/mask_ab.py 0 c2 c3 ;;
    dgemm) step dgemm 200 ipm-zoo_amd/build/sgemm_bench d ${DGEMM_R:-10752} ${DGEMM_V:-} ;;
    mixedtests) step mixedtests 400 python -u -m pytest tests/test_gpu_mixed.py tests/test_gpu_step_paths.py tests/test_gpu_graph.py -v --timeout 240 --timeout-method thread -p no:cacheprovider ;;
    newtests) step newtests 600 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_c4_batch.py -v --timeout 400 --timeout-method thread -p no:cacheprovider ;;
    kfactor) step kfactor 300 ipm-zoo_amd/build/kbench 11264 factor 384 256 512 ;;
    trace) step trace 300 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-batched --no-instrumented ;;
    c2trace) step c2trace 300 rocprofv3 --kernel-trace -d "$OUT/c2trace" -o run --output-format csv -- python bench.py --workload c2 --steps 3 --warmup 1 --no-cpu-baseline --no-batched --no-instrumented --no-configs ;;
    c2hip) step c2hip 300 rocprofv3 --hip-trace --kernel-trace -d "$OUT/c2hip" -o run --output-format csv -- python bench.py --workload c2 --steps 3 --warmup 1 --no-cpu-baseline --no-batched --no-instrumented --no-configs ;;
    counters) step counters 120 rocprofv3 -L ;;
    panel) step panel 400 python -u -m pytest tests/test_gpu_panel_forms.py tests/test_gpu_faults.py tests/test_gpu_determinism.py -v --timeout 240 --timeout-method thread -p no:cacheprovider ;;
    diagclk) step diagclk 60 ipm-zoo_amd/build/kbench 256 diagclk ;;
    chainclk_ab) for v in ${CHV:-w0 w1 w0 w1}; do step chainclk_${CN:-2560}_$v 120 ipm-zoo_amd/build/kbench_chain_$v ${CN:-2560} chainclk ${CNBO:-384}; mv "$OUT/chainclk_${CN:-2560}_$v.log" "$OUT/chainclk_${CN:-2560}_${v}_$(date +%s%N).log"; done ;;
    chainclk) step chainclk_${CN:-2560} 120 ipm-zoo_amd/build/kbench_chain ${CN:-2560} chainclk ${CNBO:-512} ;;
    graph) step graph_probe 240 python tools/dbg/graph_probe.py ${GRAPH_SIZES:-} ;;
    ktrace) step ktrace 300 rocprofv3 --kernel-trace -d "$OUT/ktrace" -o run --output-format csv -- ipm-zoo_amd/build/kbench 11264 factor 384 ;;
    *) step "$s" 600 $s ;;
  esac
done
echo ALL DONE
