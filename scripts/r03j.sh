set -e
mkdir -p gpurun_out/r03j
timeout -k 10 300 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "parity or source or fullrows or ip" > gpurun_out/r03j/gpu_tests.log 2>&1
REPS=2 bash scripts/ab_kernels.sh r03j config4 default head default+ip_group=32
REPS=2 bash scripts/ab_kernels.sh r03j config3 default head
