# MFMA counters over eager steps (one PMC pass of its own): pmc_mfma.sh OUT CONFIG
# lists the device's counters first and asks only for the MFMA ones it has (<= 6, + 2 SQ totals)
set -e
OUT=gpurun_out/$1; CFG=$2; shift 2; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
C=$(python3 - $OUT/counters_list.txt <<'EOF'
import re, sys
txt = open(sys.argv[1], errors="replace").read()
want = ["SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_MFMA", "SQ_INSTS_VALU_MFMA_I8", "SQ_INSTS_VALU_MFMA_F8",
        "SQ_INSTS_VALU_MFMA_F16", "SQ_INSTS_VALU_MFMA_BF16", "SQ_INSTS_VALU_MFMA_F32", "SQ_INSTS_VALU_MFMA_F64"]
have = [w for w in want if re.search(r"\b" + w + r"\b", txt)][:6]
print(" ".join(have + ["SQ_BUSY_CYCLES", "SQ_INSTS_VALU"]))
EOF
)
echo "counters: $C" > $OUT/mfma_$CFG.log
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/mfma_$CFG -o mfma -- python3 scripts/profile_eager.py $CFG 3 >> $OUT/mfma_$CFG.log 2>&1
