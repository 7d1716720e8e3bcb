# source-row partition: its GPU tests, then one-GPU shard scaling of both partitions and bench lines
set -e
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "source_rows_synthetic or duplicate or yaml" > $OUT/gpu_tests.log 2>&1
for c in config3 config4; do
  timeout -k 10 300 python -u scripts/partition_scaling.py $c steps=20 reps=2 > $OUT/scaling_$c.log 2>&1
done
for p in source target; do
  timeout -k 10 300 python -u bench.py --config config3 --no-cpu-baseline --steps 30 --warmup 10 --partition $p > $OUT/bench_config3_$p.log 2>&1
done
