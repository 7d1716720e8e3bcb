# Copy a measurement-set call's outputs (lease steps prof / bench / tl / scale / dist) into profiles/:
#   bash scripts/collect_profiles.sh OUT PREFIX     e.g. collect_profiles.sh r05z r05
set -e
R=gpurun_out/$1; P=profiles/$2
for c in 2 3 4 5; do [ -f $R/bench_config$c.log ] && cp $R/bench_config$c.log ${P}_bench_config$c.log; done
for c in 3 4; do
  [ -d $R/prof_config$c ] || continue
  python3 scripts/rocpd_stats.py $R/prof_config$c/run_results.db ${P}_config${c}_kernel_stats.csv > /dev/null
  python3 scripts/pmc_summary.py $(ls $R/pmc_fetch_config$c/*counter_collection.csv) $(ls $R/pmc_write_config$c/*counter_collection.csv) \
    ${P}_pmc_config$c.json config$c --mfma $(ls $R/mfma_config$c/*counter_collection.csv) --build-info $R/build_info.json > /dev/null
done
for c in 2 3 4; do
  [ -d $R/tl_config$c ] && python3 scripts/graph_timeline.py show $R/tl_config$c/run_results.db > ${P}_graph_timeline_config$c.txt
done
ls $R/scaling_*.log > /dev/null 2>&1 && grep -hv amdgpu $R/scaling_*.log > ${P}_partition_scaling.txt
for f in $R/dist_1_*.log; do [ -f "$f" ] && grep -v amdgpu "$f" > ${P}_bench_config3_rccl_world1.log; done
for f in $R/dist_2_*.log; do [ -f "$f" ] && grep -v amdgpu "$f" > ${P}_bench_config3_gloo2_rehearsal.log; done
echo "collected $R -> ${P}_*"
