set -u
export TMPDIR=/tmp
O=gpurun_out/gp
mkdir -p $O
timeout -k 10 120 ipm-zoo_amd/build/gemm_ref > $O/gemm_ref.log 2>&1 || exit $?
timeout -k 10 60 ipm-zoo_amd/build/kbench 11264 gemm > $O/kb.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS -d $O/p1 -o run --output-format csv -- ipm-zoo_amd/build/kbench 11264 gemm > $O/p1.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum -d $O/p2 -o run --output-format csv -- ipm-zoo_amd/build/kbench 11264 gemm > $O/p2.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVES -d $O/p3 -o run --output-format csv -- ipm-zoo_amd/build/kbench 11264 gemm > $O/p3.log 2>&1 || exit $?
echo done
