# C2 outer-panel width A/B on one box: tools/run_nbo.sh OUTDIR WORKLOAD NBO...
set -u
OUT=gpurun_out/$1; W=$2; shift 2; mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for nbo in "$@"; do
    AB_NBO=$nbo TORCH_STREAM=1 timeout -k 10 200 python -u tools/mask_ab.py 0 $W > $OUT/nbo_${nbo}_$i.log 2>&1 || exit 1
  done
done
for f in $OUT/nbo_*.log; do echo "$(basename $f) $(grep "^$W " $f | sed 's/.*(//' | awk '{s+=$1} END {printf "%.2f", s/NR}')"; done
