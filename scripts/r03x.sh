set -e
mkdir -p gpurun_out/r03x
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03x/gpu_tests.log 2>&1
REPS=2 bash scripts/ab_kernels.sh r03x config2 default head
REPS=2 bash scripts/ab_kernels.sh r03x config4 default head wb2 default+ip_group=32
REPS=2 bash scripts/ab_kernels.sh r03x config3 default head
