set -e
OUT=gpurun_out/r03q2; mkdir -p $OUT
export CYC_BENCH_FORCE_DIST=1
for c in config2 config3; do
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 10 --warmup 3 --config $c --no-cpu-baseline > $OUT/rccl_world1_$c.log 2>&1
done
