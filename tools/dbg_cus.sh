set -o pipefail
O=gpurun_out/${OUTD:-r05_s29}; mkdir -p $O
for v in "" 113 128; do
  timeout -k 10 100 ipm-zoo_amd/build/kbench_chain$v 11264 chainclk 512 > $O/chain11264_$v.log 2>&1 || exit 1
  timeout -k 10 60 ipm-zoo_amd/build/kbench_chain$v 2560 chainclk 512 > $O/chain2560_$v.log 2>&1 || exit 1
done
grep -H "factor N" $O/*.log
