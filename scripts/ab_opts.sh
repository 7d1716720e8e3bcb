# A/B of cyc_set_option settings on one box: ab_opts.sh OUT CONFIG "opt1=v opt2=v" "..." (empty string = defaults)
set -e
OUT=gpurun_out/$1; CFG=$2; shift 2; mkdir -p $OUT
for rep in 1 2; do
i=0
for spec in "$@"; do
  i=$((i+1)); args=""
  for o in $spec; do args="$args --opt $o"; done
  timeout -k 10 300 python -u bench.py --config $CFG --no-cpu-baseline --steps 30 --warmup 10 $args > $OUT/opt_${CFG}_${i}_$rep.log 2>&1
  echo "$i: $spec" > $OUT/opt_${CFG}_${i}.spec
done
done
