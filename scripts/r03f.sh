set -e
OUT=gpurun_out/r03f; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or source or dist or pod_words or fullrows" > $OUT/gpu_tests.log 2>&1
REPS=2 bash scripts/ab_kernels.sh r03f config3 default prev pbh8
REPS=2 bash scripts/ab_kernels.sh r03f config4 default prev mb1 mb4
export CYC_SHARD=0/8
CYC_PART=source bash scripts/ab_kernels.sh r03f_src8 config3 default prev
CYC_PART=target bash scripts/ab_kernels.sh r03f_tgt8 config3 default prev
