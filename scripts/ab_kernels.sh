# kernel stats of eager steps per library variant: ab_kernels.sh OUT CFG VAR... (default | var name)
set -e
OUT=gpurun_out/$1; CFG=$2; shift 2; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in "$@"; do
  if [ "$v" = default ]; then LIB=""; else LIB=cyclonus_amd/_build/var_$v/libcyclonus_hip.so; fi
  CYC_HIP_LIB=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/k_${CFG}_$v -o run -- python3 scripts/profile_eager.py $CFG 20 > $OUT/k_${CFG}_$v.log 2>&1
done
