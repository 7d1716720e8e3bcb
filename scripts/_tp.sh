set -e
OUT=gpurun_out/$1; mkdir -p $OUT
for cus in 16 32 64; do
timeout -k 10 200 python -u scripts/throughput.py config3 init.front_cus=$cus pipelined=0,1 front_graph=0,1 >> $OUT/tp.log 2>&1
timeout -k 10 200 python -u scripts/throughput.py config3 init.front_cus=$cus pipelined=0,1 front_graph=0,1 shards=8 >> $OUT/tp.log 2>&1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace -d $OUT/c3s8p -o run -- python3 scripts/throughput.py config3 init.front_cus=32 pipelined=1 reps=1 steps=10 shards=8 >> $OUT/tl.log 2>&1
