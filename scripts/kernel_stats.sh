# per-kernel stats of eager steps: kernel_stats.sh OUT CONFIG [NAME=VALUE ...]
set -e
OUT=gpurun_out/$1; CFG=$2; shift 2; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAG=$(echo "$CFG $@" | tr ' =' '__')
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run -- python3 scripts/profile_eager.py $CFG 20 "$@" > $OUT/prof_$TAG.log 2>&1
