# iteration: GPU tests, then bench + kernel stats of the configs given
set -e
OUT=gpurun_out/$1; shift; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in "$@"; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $OUT/bench_$c.log 2>&1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run -- python3 scripts/profile_eager.py $c 20 > $OUT/prof_$c.log 2>&1
done
