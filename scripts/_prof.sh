# Round-end measurement set for one config: bench line, rocprofv3 --kernel-trace --stats of the
# same bench command, and separate FETCH_SIZE / WRITE_SIZE / MFMA PMC passes over eager steps
# (summarise here with scripts/pmc_summary.py ... --mfma ...).
#   bash scripts/_prof.sh OUTDIR config3
set -e
OUT=gpurun_out/$1; CFG=$2; mkdir -p $OUT
cp cyclonus_amd/_build/build_info.json $OUT/build_info.json
timeout -k 10 300 python -u bench.py --config $CFG > $OUT/bench_$CFG.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$CFG -o run -- python3 bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof_$CFG.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_$CFG -o fetch -- python3 scripts/profile_eager.py $CFG 5 > $OUT/pmc_fetch_$CFG.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_$CFG -o write -- python3 scripts/profile_eager.py $CFG 5 > $OUT/pmc_write_$CFG.log 2>&1
bash scripts/pmc_mfma.sh $1 $CFG
