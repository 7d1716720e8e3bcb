set -e
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 200 python -u scripts/throughput.py config2 graphs=0,1 graph_branches=0,1 >> $OUT/tp.log 2>&1
timeout -k 10 200 python -u scripts/throughput.py config3 graphs=0,1 graph_branches=0,1 shards=8 >> $OUT/tp.log 2>&1
timeout -k 10 200 python -u scripts/throughput.py config4 graphs=0,1 graph_branches=0,1 >> $OUT/tp.log 2>&1
timeout -k 10 200 python -u scripts/throughput.py config3 graphs=0,1 graph_branches=0,1 >> $OUT/tp.log 2>&1
