# fused-front A/B: GPU tests, step throughput by option, graph timelines
set -e
OUT=gpurun_out/$1; shift; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
for spec in "$@"; do timeout -k 10 200 python -u scripts/throughput.py $spec >> $OUT/tp.log 2>&1; done
