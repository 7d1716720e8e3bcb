set -e
OUT=gpurun_out/r03r2; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullrows.py -k "direct or config2 or random_parity or random_panics or launch_modes or source_rows_synthetic" -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
REPS=2 bash scripts/ab_kernels.sh r03r2 config2 default g1 g8
