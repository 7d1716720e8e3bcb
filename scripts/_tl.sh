# graph timelines (rocprofv3 kernel trace of graph replays) for the configs given
set -e
OUT=gpurun_out/$1; shift; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for spec in "$@"; do
  tag=$(echo $spec | tr ' =' '__')
  timeout -k 10 120 rocprofv3 --kernel-trace -d $OUT/$tag -o run -- python3 scripts/graph_timeline.py run $spec >> $OUT/tl.log 2>&1
done
