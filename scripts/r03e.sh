set -e
OUT=gpurun_out/r03e; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
for c in config3 config4; do
  timeout -k 10 300 python -u scripts/partition_scaling.py $c steps=20 reps=2 > $OUT/scaling_$c.log 2>&1
done
export CYC_SHARD=0/8
CYC_PART=source bash scripts/ab_kernels.sh r03e_src8 config3 default
CYC_PART=target bash scripts/ab_kernels.sh r03e_tgt8 config3 default
