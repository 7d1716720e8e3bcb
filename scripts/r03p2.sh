set -e
OUT=gpurun_out/r03p2; mkdir -p $OUT
REPS=2 bash scripts/ab_kernels.sh r03p2 config3 default efuse
for i in 1 2; do
timeout -k 10 300 python -u bench.py --config config3 --no-cpu-baseline --steps 30 --warmup 10 > $OUT/bench_default_$i.log 2>&1
CYC_HIP_LIB=cyclonus_amd/_build/var_efuse/libcyclonus_hip.so timeout -k 10 300 python -u bench.py --config config3 --no-cpu-baseline --steps 30 --warmup 10 > $OUT/bench_efuse_$i.log 2>&1
done
CYC_HIP_LIB=cyclonus_amd/_build/var_efuse/libcyclonus_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "uniform or random_parity or launch_modes" -x -q --timeout 120 --timeout-method thread > $OUT/tests_efuse.log 2>&1
