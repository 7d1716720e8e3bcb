set -e
REPS=2 bash scripts/ab_kernels.sh r03m config3 default noip noexp idonostore
