# SQ instruction-mix counters per kernel over eager steps (one --pmc pass, <= 8 SQ counters)
set -e
OUT=gpurun_out/$1; CFG=$2; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_ANY --output-format csv -d $OUT/sq_$CFG -o sq -- python3 scripts/profile_eager.py $CFG 3 > $OUT/sq_$CFG.log 2>&1
