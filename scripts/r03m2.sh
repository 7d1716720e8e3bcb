set -e
bash scripts/_final3.sh r03g
OUT=gpurun_out/r03g
for i in 1 2; do
timeout -k 10 300 python -u bench.py --config config3 --no-cpu-baseline --steps 30 --warmup 10 > $OUT/ab_default_$i.log 2>&1
CYC_HIP_LIB=cyclonus_amd/_build/var_e512/libcyclonus_hip.so timeout -k 10 300 python -u bench.py --config config3 --no-cpu-baseline --steps 30 --warmup 10 > $OUT/ab_e512_$i.log 2>&1
done
REPS=2 bash scripts/ab_kernels.sh r03g config4 default pipe
