set -e
mkdir -p gpurun_out/r03h
timeout -k 10 400 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu -k "uniform or parity or source or fullrows or pod_words or table or dist or batch" > gpurun_out/r03h/gpu_tests.log 2>&1
REPS=2 bash scripts/ab_kernels.sh r03h config3 default nouni
REPS=2 bash scripts/ab_kernels.sh r03h config4 default nouni
