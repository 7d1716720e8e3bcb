set -e
mkdir -p gpurun_out/r03v
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03v/gpu_tests.log 2>&1
REPS=2 bash scripts/ab_kernels.sh r03v config4 default head
REPS=2 bash scripts/ab_kernels.sh r03v config3 default head
REPS=2 bash scripts/ab_kernels.sh r03v config2 default head
