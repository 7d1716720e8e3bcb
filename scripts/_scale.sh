# strong-scaling prediction on one GPU: back-to-back step time of rank 0's row shard for N = 1, 2, 4, 8
set -e
OUT=gpurun_out/$1; mkdir -p $OUT
for n in 1 2 4 8; do
  timeout -k 10 200 python -u scripts/throughput.py config3 shards=$n reps=2 >> $OUT/scale.log 2>&1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace -d $OUT/tl3 -o run -- python3 scripts/graph_timeline.py run config3 10 > $OUT/tl.log 2>&1
