set -e
REPS=2 bash scripts/ab_kernels.sh r03l config4 default noload nostore wb16 onechunk
