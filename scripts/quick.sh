# quick perf check: bench (2 reps) + kernel stats for each config given
set -e
OUT=gpurun_out/$1; shift; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in "$@"; do
  for rep in 1 2; do timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --steps 30 --warmup 10 > $OUT/bench_${c}_$rep.log 2>&1; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run -- python3 scripts/profile_eager.py $c 20 > $OUT/prof_$c.log 2>&1
done
