# config #4 front study: kernel stats fused / two-branch DAG, SQ passes of both
set -e
bash scripts/prof_front.sh r03i config4
OUT=gpurun_out/r03i
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P="python3 scripts/profile_eager.py config4 3 front_fused=0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $OUT/sq1dag_config4 -o sq1 -- $P > $OUT/sq1dag.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/sq2dag_config4 -o sq2 -- $P > $OUT/sq2dag.log 2>&1
