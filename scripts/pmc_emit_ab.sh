# Emit PMC passes per emit_halves_ab.py variant (each pass its own run, all variants in one process):
#   pmc_emit_ab.sh OUT VARIANT...   -> gpurun_out/OUT/pmcab_<pass>/..., summary pmcab_summary.txt
set -e
OUT=gpurun_out/$1; shift; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P="python3 scripts/emit_halves_ab.py run $* n=3"
pass() {  # pass NAME COUNTERS...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $OUT/pmcab_$name -o $name -- $P > $OUT/pmcab_$name.log 2>&1
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum
pass tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum
pass lvl TCC_TAG_STALL_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_sum
pass utcl TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_SERIALIZATION_STALL_sum
pass utcl2 TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_UTCL1_STALL_MULTI_MISS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE
pass ta TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE
python3 scripts/pmc_emit_ab.py $OUT "$@" > $OUT/pmcab_summary.txt 2>&1
