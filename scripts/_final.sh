# round-end measurement set: GPU tests, smoke, bench lines (configs 3, 2, 4, 5), rocprof stats + PMC
# (FETCH / WRITE / MFMA) of configs 3 and 4, scaling prediction and graph timeline
set -e
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
bash scripts/_prof.sh $1 config3
bash scripts/_prof.sh $1 config4
for c in config2 config5; do timeout -k 10 300 python -u bench.py --config $c > $OUT/bench_$c.log 2>&1; done
bash scripts/_scale.sh $1
