set -e
OUT=gpurun_out/r03o2; mkdir -p $OUT
for p in target source; do timeout -k 10 300 python -u scripts/throughput.py config3 shards=8 part=$p reps=2 >> $OUT/tp.log 2>&1; done
for p in target source; do timeout -k 10 300 python -u scripts/throughput.py config3 shards=2 part=$p reps=2 >> $OUT/tp.log 2>&1; done
