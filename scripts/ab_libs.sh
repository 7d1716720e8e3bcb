# A/B of library variants on one box: ab_libs.sh OUT CONFIG VARIANT... (VARIANT = default | name of _build/var_NAME)
set -e
OUT=gpurun_out/$1; CFG=$2; shift 2; mkdir -p $OUT
for rep in 1 2; do
for v in "$@"; do
  if [ "$v" = default ]; then LIB=""; else LIB=cyclonus_amd/_build/var_$v/libcyclonus_hip.so; fi
  CYC_HIP_LIB=$LIB timeout -k 10 300 python -u bench.py --config $CFG --no-cpu-baseline --steps 30 --warmup 10 > $OUT/ab_${CFG}_${v}_$rep.log 2>&1
done
done
