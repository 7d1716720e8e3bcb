# per-rank step time of every row shard of an N-way run on one GPU (load balance across ranks)
set -e
OUT=gpurun_out/$1; N=$2; CFG=${3:-config3}; mkdir -p $OUT
for r in $(seq 0 $((N - 1))); do
  timeout -k 10 200 python -u scripts/throughput.py $CFG shards=$N rank=$r reps=2 >> $OUT/ranks.log 2>&1
done
