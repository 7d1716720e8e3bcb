# Round-3 measurement set, the essentials (GPU tests, smoke, bench line + rocprofv3 stats + PMC of configs 3 and 4,
# bench lines of configs 2 and 5):  bash scripts/_final3_min.sh OUT
set -e
NAME=$1; OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
bash scripts/_prof.sh $NAME config3
bash scripts/_prof.sh $NAME config4
for c in config2 config5; do timeout -k 10 300 python -u bench.py --config $c > $OUT/bench_$c.log 2>&1; done
