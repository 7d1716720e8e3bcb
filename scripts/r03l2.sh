set -e
OUT=gpurun_out/r03l2; mkdir -p $OUT
for i in 1 2; do
for v in default e1024 e512x7 ewaves; do
  if [ $v = default ]; then LIB=""; else LIB=cyclonus_amd/_build/var_$v/libcyclonus_hip.so; fi
  CYC_HIP_LIB=$LIB timeout -k 10 300 python -u bench.py --config config3 --no-cpu-baseline --steps 30 --warmup 10 > $OUT/bench_${v}_$i.log 2>&1
done
done
REPS=1 bash scripts/ab_kernels.sh r03l2 config4 default ewaves
