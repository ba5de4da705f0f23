set -o pipefail
O=gpurun_out/${OUTD:-r05_pmc3}; mkdir -p $O
for w in c2 c3 c5; do
  PMCW=$w OUT=$O STEPS="pmcf_fetch pmcf_write pmcf_mops pmcf_busy" bash tools/gpu_round.sh || exit 1
done
