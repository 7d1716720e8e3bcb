# GPU tests, then per config: kernel stats of eager steps (ab_kernels.sh SPECS, default "default")
# and a bench line:  check.sh OUT "CFG..." [SPEC...]
set -e
NAME=$1; OUT=gpurun_out/$1; CFGS=$2; shift 2; SPECS=${@:-default}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in $CFGS; do
  bash scripts/ab_kernels.sh $NAME $c $SPECS
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --steps 30 --warmup 10 > $OUT/bench_$c.log 2>&1
done
