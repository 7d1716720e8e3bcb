# GPU test suite (optionally a -k filter), then a config3 + config4 bench line:  gputest.sh OUT [-k EXPR]
set -e
OUT=gpurun_out/$1; shift; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > $OUT/gpu_tests.log 2>&1
for c in config3 config4; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --steps 30 --warmup 10 > $OUT/bench_$c.log 2>&1
done
