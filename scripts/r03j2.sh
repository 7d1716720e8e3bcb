set -e
OUT=gpurun_out/r03j2; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullrows.py tests/test_gpu_table.py tests/test_gpu_api.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
REPS=2 bash scripts/ab_kernels.sh r03j2 config3 default notab
REPS=2 bash scripts/ab_kernels.sh r03j2 config4 default notab
timeout -k 10 300 python -u bench.py --config config3 --no-cpu-baseline --steps 30 --warmup 10 > $OUT/bench_config3.log 2>&1
CYC_HIP_LIB=cyclonus_amd/_build/var_notab/libcyclonus_hip.so timeout -k 10 300 python -u bench.py --config config3 --no-cpu-baseline --steps 30 --warmup 10 > $OUT/bench_config3_notab.log 2>&1
