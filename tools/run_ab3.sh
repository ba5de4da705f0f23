# A/B/C of package builds on one box: tools/run_ab3.sh OUTDIR WORKLOADS VARIANT_DIR...
# (each variant: a package directory, "." = this tree)
set -u
OUT=gpurun_out/$1; W=$2; shift 2; mkdir -p $OUT
export TMPDIR=/tmp
for i in ${REPS:-1 2}; do
  for v in "$@"; do
    n=$(echo $v | tr '/.' '__')
    if [ "$v" = "." ]; then d=""; else d=$v/ipm-zoo_amd; fi
    TORCH_STREAM=1 IPMZ_PKG_DIR=$d timeout -k 10 200 python -u tools/mask_ab.py 0 $W > $OUT/ab_${n}_$i.log 2>&1 || exit 1
  done
done
for f in $OUT/ab_*.log; do
  for w in $W; do echo "$(basename $f) $w $(grep "^$w " $f | sed 's/.*(//' | awk '{s+=$1} END {printf "%.2f", s/NR}')"; done
done
