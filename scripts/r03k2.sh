set -e
OUT=gpurun_out/r03k2; mkdir -p $OUT
timeout -k 10 120 ./scripts/wbw 20 > $OUT/wbw.txt 2>&1
for i in 1 2; do
timeout -k 10 300 python -u bench.py --config config3 --no-cpu-baseline --steps 30 --warmup 10 > $OUT/bench_default_$i.log 2>&1
CYC_HIP_LIB=cyclonus_amd/_build/var_tab/libcyclonus_hip.so timeout -k 10 300 python -u bench.py --config config3 --no-cpu-baseline --steps 30 --warmup 10 > $OUT/bench_tab_$i.log 2>&1
done
