set -e
OUT=gpurun_out/r02_base; mkdir -p $OUT
timeout -k 10 300 python -u bench.py --config config4 --no-cpu-baseline > $OUT/bench_config4.log 2>&1
timeout -k 10 300 python -u bench.py --config config3 --no-cpu-baseline > $OUT/bench_config3.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof4 -o run -- python3 scripts/profile_eager.py config4 20 > $OUT/prof4.log 2>&1
