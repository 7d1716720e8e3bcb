set -e
OUT=gpurun_out/r03g2; mkdir -p $OUT
for i in 1 2; do timeout -k 10 300 python -u bench.py --config config3 --no-cpu-baseline --steps 30 --warmup 10 > $OUT/bench_config3_$i.log 2>&1; done
PYTORCH_NO_HIP_MEMORY_CACHING=1 timeout -k 10 300 python -u bench.py --config config3 --no-cpu-baseline --steps 30 --warmup 10 > $OUT/bench_config3_nocache.log 2>&1
timeout -k 10 300 python -u scripts/throughput.py config3 reps=3 > $OUT/throughput_config3.log 2>&1
REPS=2 bash scripts/ab_kernels.sh r03g2 config3 default ipskip
