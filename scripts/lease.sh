# One parametrised GPU call: every step runs under its own time limit, results under gpurun_out/OUT/,
# and the first failing step ends the call (set -e; no GPU step runs after a fault or a timeout).
#   gpurun -- 'bash scripts/lease.sh OUT "tests [-k EXPR]" "smoke" "bench CFG [bench args]" ...'
# steps:
#   tests [pytest args]        GPU test suite (-m gpu; K=a+or+b selects -k "a or b")
#   smoke                      __graft_entry__.smoke()
#   bench CFG [args]           python bench.py --config CFG [args]       -> bench_CFG[_TAG].log
#   prof CFG                   bench line, rocprofv3 --kernel-trace --stats of the bench command,
#                              FETCH_SIZE / WRITE_SIZE / MFMA PMC passes over eager steps
#   ks CFG N [NAME=V ...]      kernel stats of N eager steps (tokens CYC_SHARD=r/N, CYC_PART=source|target)
#   scale CFG                  scripts/partition_scaling.py (one-GPU shard timings, both partitions)
#   tl CFG [N]                 kernel timeline of back-to-back steps (scripts/graph_timeline.py)
#   py SCRIPT [args]           any python script under scripts/ (180 s limit)
#   counters                   rocprofv3 -L (the counters this box's gfx950 offers)
#   bin PROBE [args]           a probe built from scripts/*.hip (scripts/PROBE, 180 s limit)
#   dist N CFG [args]          bench.py as an N-rank torch.distributed.run job on this box (tokens:
#                              CYC_BENCH_BACKEND=gloo for a one-GPU rehearsal, CYC_BENCH_FORCE_DIST=1)
#   ab CFG SPEC...             kernel stats per library variant (scripts/ab_kernels.sh; REPS env, CYC_SHARD tokens)
#   pmcab VARIANT...           emit PMC passes per scripts/emit_halves_ab.py variant (scripts/pmc_emit_ab.sh)
#   emitks VARIANT:LAUNCHES... per-launch emit durations of emit_halves_ab.py variants (scripts/emit_launches.py)
#   pmc CFG [NAME=V ...]       per-kernel SQ instruction / wait mix, TCC hits, FETCH / WRITE passes (scripts/pmc_passes.sh)
# Invocations are recorded in scripts/LEASES.md.
set -e
NAME=$1; shift
OUT=gpurun_out/$NAME; mkdir -p $OUT
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cp cyclonus_amd/_build/build_info.json $OUT/build_info.json 2>/dev/null || true
prof_env() { cd /tmp && export TMPDIR=/tmp && cd $ROOT; }
for spec in "$@"; do
  set -- $spec
  step=$1; shift
  # CYC_*=value and REPS=n tokens are environment for this step only (e.g. "ks config3 CYC_SHARD=0/8")
  envs=(); args=()
  for a in "$@"; do if [[ $a == CYC_*=* || $a == REPS=* ]]; then envs+=("$a"); else args+=("$a"); fi; done
  set -- "${args[@]}"
  for e in "${envs[@]}"; do export "$e"; done
  tag=$(echo "$*" | tr ' =/' '___' | cut -c1-60)
  [ -n "$CYC_HIP_LIB" ] && tag=${tag}_$(basename $(dirname $CYC_HIP_LIB))  # library variant runs apart
  echo "[lease] $(date +%T) $spec" >> $OUT/steps.log
  case $step in
    tests)  # (K=a+or+b: pytest -k "a or b" — a step's words cannot hold spaces)
      targs=(); for a in "$@"; do if [[ $a == K=* ]]; then targs+=(-k "$(echo "${a#K=}" | tr '+' ' ')"); else targs+=("$a"); fi; done
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --durations=40 --timeout 300 --timeout-method thread "${targs[@]}" > $OUT/gpu_tests.log 2>&1 ;;
    smoke) timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 ;;
    bench) timeout -k 10 300 python -u bench.py --config "$@" > $OUT/bench_$tag.log 2>&1 ;;
    prof)
      CFG=$1
      timeout -k 10 300 python -u bench.py --config $CFG > $OUT/bench_$CFG.log 2>&1
      prof_env
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$CFG -o run -- python3 bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof_$CFG.log 2>&1
      timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_$CFG -o fetch -- python3 scripts/profile_eager.py $CFG 5 > $OUT/pmc_fetch_$CFG.log 2>&1
      timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_$CFG -o write -- python3 scripts/profile_eager.py $CFG 5 > $OUT/pmc_write_$CFG.log 2>&1
      bash scripts/pmc_mfma.sh $NAME $CFG ;;
    ks)
      prof_env
      sfx=$(echo "${CYC_SHARD:+_$CYC_SHARD}${CYC_PART:+_$CYC_PART}" | tr / of)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ks_$tag$sfx -o run -- python3 scripts/profile_eager.py "$@" > $OUT/ks_$tag$sfx.log 2>&1 ;;
    scale) timeout -k 10 400 python -u scripts/partition_scaling.py "$@" > $OUT/scaling_$tag.log 2>&1 ;;
    tl)
      prof_env
      timeout -k 10 120 rocprofv3 --kernel-trace -d $OUT/tl_$tag -o run -- python3 scripts/graph_timeline.py run "$@" > $OUT/tl_$tag.log 2>&1 ;;
    py) timeout -k 10 180 python -u scripts/"$@" > $OUT/py_$tag.log 2>&1 ;;
    counters) prof_env; timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 ;;
    bin) timeout -k 10 180 ./scripts/"$@" > $OUT/bin_$tag.log 2>&1 ;;
    dist)
      NP=$1; CFG=$2; shift 2
      timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $NP --master-addr 127.0.0.1 \
        --master-port $((29500 + RANDOM % 400)) bench.py --gpus $NP --config $CFG "$@" > $OUT/dist_$tag.log 2>&1 ;;
    ab) timeout -k 10 900 bash scripts/ab_kernels.sh $NAME "$@" ;;
    pmc) timeout -k 10 700 bash scripts/pmc_passes.sh $NAME "$@" ;;
    pmcab) timeout -k 10 900 bash scripts/pmc_emit_ab.sh $NAME "$@" ;;
    emitks)  # per-launch emit durations of emit_halves_ab.py variants (VARIANT:LAUNCHES ...), kernel trace
      prof_env
      vs=(); for a in "$@"; do vs+=("${a%%:*}"); done
      timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/emitks -o run -- python3 scripts/emit_halves_ab.py run "${vs[@]}" n=10 > $OUT/emitks.log 2>&1
      python3 scripts/emit_launches.py $OUT/emitks/run_results.db "$@" n=10 > $OUT/emitks_summary.txt 2>&1 ;;
    *) echo "unknown step $step" >&2; exit 2 ;;
  esac
  for e in "${envs[@]}"; do unset "${e%%=*}"; done
done
echo "[lease] $(date +%T) done" >> $OUT/steps.log
