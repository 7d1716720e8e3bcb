# kernel stats of eager steps per library variant, interleaved over REPS rounds:
#   ab_kernels.sh OUT CFG SPEC...   SPEC = default | NAME (of _build/var_NAME) [+opt=v[+opt=v]]
# (REPS env, default 1: each round runs every spec once, so box drift hits all specs alike)
set -e
OUT=gpurun_out/$1; CFG=$2; shift 2; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in $(seq 1 ${REPS:-1}); do
  for spec in "$@"; do
    v=${spec%%+*}; opts=""
    [ "$spec" != "$v" ] && opts=$(echo "${spec#*+}" | tr '+' ' ')
    if [ "$v" = default ]; then LIB=""; else LIB=cyclonus_amd/_build/var_$v/libcyclonus_hip.so; fi
    tag=$(echo "$spec" | tr '+=' '__'); [ "${REPS:-1}" -gt 1 ] && tag=${tag}_r$r
    tag=${tag}$(echo "${CYC_SHARD:+_s$CYC_SHARD}${CYC_PART:+_$CYC_PART}" | tr / o)
    tag=${tag}${CYC_DBG_BKEEP:+_k$CYC_DBG_BKEEP}  # timing-probe variants (launch B ranges kept)
    CYC_HIP_LIB=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/k_${CFG}_$tag -o run -- python3 scripts/profile_eager.py $CFG 20 $opts > $OUT/k_${CFG}_$tag.log 2>&1
  done
done
