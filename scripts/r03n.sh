set -e
mkdir -p gpurun_out/r03n
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "parity or fullrows or pl or batch or table or ido or source" > gpurun_out/r03n/gpu_tests.log 2>&1
REPS=2 bash scripts/ab_kernels.sh r03n config4 default head flat2 flat4
REPS=2 bash scripts/ab_kernels.sh r03n config3 default head
