set -e
mkdir -p gpurun_out/r03k
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "parity or fullrows or pl or batch or table or ido" > gpurun_out/r03k/gpu_tests.log 2>&1
REPS=2 bash scripts/ab_kernels.sh r03k config4 default head nochunk onechunk t256
REPS=2 bash scripts/ab_kernels.sh r03k config3 default head
