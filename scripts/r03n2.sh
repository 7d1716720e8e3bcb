set -e
for n in 2 8; do
  CYC_SHARD=0/$n CYC_PART=source REPS=1 bash scripts/ab_kernels.sh r03n2_src$n config3 default
  CYC_SHARD=0/$n CYC_PART=target REPS=1 bash scripts/ab_kernels.sh r03n2_tgt$n config3 default
done
