set -e
OUT=gpurun_out/r03t2; mkdir -p $OUT
CYC_HIP_LIB=cyclonus_amd/_build/var_cistage/libcyclonus_hip.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests_cistage.log 2>&1
REPS=2 bash scripts/ab_kernels.sh r03t2 config3 default cistage
