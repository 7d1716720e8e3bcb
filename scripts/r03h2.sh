set -e
REPS=2 bash scripts/ab_kernels.sh r03h2 config3 default enoload elinear eboth
REPS=2 bash scripts/ab_kernels.sh r03h2 config4 default enoload elinear
