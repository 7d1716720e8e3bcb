set -e
REPS=2 bash scripts/ab_kernels.sh r03g config3 default cig8
REPS=2 bash scripts/ab_kernels.sh r03g config4 default plpair
export CYC_SHARD=0/8
CYC_PART=source REPS=2 bash scripts/ab_kernels.sh r03g_src8 config3 default cig8
CYC_PART=source REPS=2 bash scripts/ab_kernels.sh r03g_src8 config4 default plpair
