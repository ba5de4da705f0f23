# debug-bit A/B on one box: tools/run_mask.sh OUTDIR MASK WORKLOADS
set -u
OUT=gpurun_out/$1; M=$2; W=$3; mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2 3; do
  TORCH_STREAM=1 timeout -k 10 200 python -u tools/mask_ab.py $M $W > $OUT/mask_$i.log 2>&1 || exit 1
done
for w in $W; do for m in 0 $M; do echo "$w mask $m: $(cat $OUT/mask_*.log | grep "^$w mask $m:" | sed 's/.*(//' | awk '{s+=$1} END {printf "%.2f (n=%d)", s/NR, NR}')"; done; done
