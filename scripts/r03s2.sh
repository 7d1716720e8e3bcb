set -e
OUT=gpurun_out/r03s2; mkdir -p $OUT
timeout -k 10 120 ./scripts/wbw 20 > $OUT/wbw.txt 2>&1
REPS=2 bash scripts/ab_kernels.sh r03s2 config3 default enoload etab
REPS=2 bash scripts/ab_kernels.sh r03s2 config4 default enoload etab
