# Round-3 measurement set on the final build (one box, one call):
#   GPU tests, smoke, bench line + rocprofv3 stats + PMC (FETCH / WRITE / MFMA) for configs 3 and 4,
#   bench lines of configs 2 and 5, both partitions' one-GPU shard scaling (config #3), a step timeline.
#   bash scripts/_final3.sh OUT
set -e
NAME=$1; OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
bash scripts/_prof.sh $NAME config3
bash scripts/_prof.sh $NAME config4
for c in config2 config5; do timeout -k 10 300 python -u bench.py --config $c > $OUT/bench_$c.log 2>&1; done
timeout -k 10 400 python -u scripts/partition_scaling.py config3 steps=20 reps=2 > $OUT/scaling_config3.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace -d $OUT/tl3 -o run -- python3 scripts/graph_timeline.py run config3 10 > $OUT/tl.log 2>&1
