set -e
mkdir -p gpurun_out/r03z
REPS=2 bash scripts/ab_kernels.sh r03z config3 default grp4 grp8 plain grp8p
REPS=2 bash scripts/ab_kernels.sh r03z config4 default grp4 grp8 plain grp8p
CYC_HIP_LIB=cyclonus_amd/_build/var_grp8/libcyclonus_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_fullrows.py tests/test_gpu_table.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03z/tests_grp8.log 2>&1
