set -e
mkdir -p gpurun_out/r03y
timeout -k 10 120 ./scripts/wbw 20 > gpurun_out/r03y/wbw.txt 2>&1
REPS=3 bash scripts/ab_kernels.sh r03y config2 default noskip head
