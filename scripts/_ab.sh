# A/B of two library builds (CYC_HIP_LIB) on the same box: graph / eager step times per config
#   bash scripts/_ab.sh OUTDIR "config3 config4" "emit_variant=0,7,8"
set -e
OUT=gpurun_out/$1; mkdir -p $OUT
PREV=cyclonus_amd/_build/libcyclonus_hip_prev.so
for cfg in $2; do
  for lib in new prev; do
    if [ $lib = prev ]; then export CYC_HIP_LIB=$PREV; ARGS="emit_variant=0"; else unset CYC_HIP_LIB; ARGS="$3"; fi
    echo "== $cfg $lib" >> $OUT/ab.log
    timeout -k 10 200 python -u scripts/opt_sweep.py $cfg $ARGS reps=3 >> $OUT/ab.log 2>&1
  done
done
