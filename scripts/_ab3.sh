# throughput A/B of the current build vs cyclonus_amd/_build/libcyclonus_hip_prev.so
set -e
OUT=gpurun_out/$1; shift; mkdir -p $OUT
PREV=cyclonus_amd/_build/libcyclonus_hip_prev.so
for spec in "$@"; do
  for lib in new prev new prev; do
    if [ $lib = prev ]; then export CYC_HIP_LIB=$PREV; else unset CYC_HIP_LIB; fi
    echo "== $spec $lib" >> $OUT/ab.log
    timeout -k 10 200 python -u scripts/throughput.py $spec reps=2 >> $OUT/ab.log 2>&1
  done
done
