set -e
mkdir -p gpurun_out/r03u
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03u/gpu_tests.log 2>&1
REPS=2 bash scripts/ab_kernels.sh r03u config4 default head nopipe
REPS=2 bash scripts/ab_kernels.sh r03u config3 default head pf cpb2pf
