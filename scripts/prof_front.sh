# front-kernel study for one config: kernel stats of eager steps on the fused front and on the
# two-branch DAG (one kernel per stage), then SQ counter passes of the fused front
#   bash scripts/prof_front.sh OUT CFG [NAME=VALUE ...]
set -e
OUT=gpurun_out/$1; CFG=$2; shift 2; mkdir -p $OUT
cp cyclonus_amd/_build/build_info.json $OUT/build_info.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/ks_$CFG -o run -- python3 scripts/profile_eager.py $CFG 10 "$@" > $OUT/ks_$CFG.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/ksdag_$CFG -o run -- python3 scripts/profile_eager.py $CFG 10 front_fused=0 "$@" > $OUT/ksdag_$CFG.log 2>&1
P="python3 scripts/profile_eager.py $CFG 3 $@"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $OUT/sq1_$CFG -o sq1 -- $P > $OUT/sq1_$CFG.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/sq2_$CFG -o sq2 -- $P > $OUT/sq2_$CFG.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/tcc_$CFG -o tcc -- $P > $OUT/tcc_$CFG.log 2>&1
