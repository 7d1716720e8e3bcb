set -e
OUT=gpurun_out/r03d; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "batch or config5 or yaml or duplicate or source_rows_synthetic" > $OUT/gpu_tests.log 2>&1
timeout -k 10 300 python -u bench.py --config config5 --no-cpu-baseline --steps 30 --warmup 10 > $OUT/bench_config5.log 2>&1
bash scripts/ab_libs.sh r03d config3 default esplit
REPS=2 bash scripts/ab_kernels.sh r03d config3 default esplit
export CYC_SHARD=0/8
CYC_PART=source bash scripts/ab_kernels.sh r03d_src8 config3 default wide8k
CYC_PART=target bash scripts/ab_kernels.sh r03d_tgt8 config3 default
