set -e
REPS=2 bash scripts/ab_kernels.sh r03w config4 default pair wb4 mix4 mix1 default+ip_group=8 default+ip_group=32
bash scripts/kernel_stats.sh r03w config4 front_fused=0
