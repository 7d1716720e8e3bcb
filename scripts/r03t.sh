set -e
bash scripts/kernel_stats.sh r03t config4 front_fused=0
bash scripts/kernel_stats.sh r03t config3 front_fused=0
REPS=2 bash scripts/ab_kernels.sh r03t config3 default cpb2 cpb4 cpb7 pf cpb2pf cpb4pf default+class_rpb=2
bash scripts/pmc_passes.sh r03t config4
