# PMC at the channel sweep's throughput end (65536 channels, one 20-epoch launch with records): one counter group
# per rocprofv3 pass, kernel-trace only (MI355X_MICROARCH.md rocprofv3 rules).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r05pmc_sweep
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 python3 $R/scripts/trk_sweep_point.py 65536 20 records > $OUT/plain.txt 2>&1 || { echo "plain run failed"; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 $R/scripts/trk_sweep_point.py 65536 20 records > $OUT/stats.txt 2>&1 || { echo "stats run failed"; exit 1; }
find $OUT/stats -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
for f in $(find $OUT/stats -name "*kernel_trace.csv"); do { head -1 $f; grep trk_ $f || true; } > $OUT/kernel_trace_trk.csv; done
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 $R/scripts/trk_sweep_point.py 65536 20 records > $OUT/p$i.txt 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
cd $R && python3 scripts/pmc_traffic.py $OUT trk_ last > $OUT/summary.json && cat $OUT/summary.json
# keep only the tracking kernel's counter rows (the merge back is size-limited)
for f in $(find $OUT -name "*counter_collection.csv"); do
  d=$(dirname $f); p=$(echo $f | sed "s#$OUT/##" | cut -d/ -f1)
  { head -1 $f; grep "trk_" $f || true; } > $OUT/${p}_trk_counters.csv
done
find $OUT -mindepth 1 -type d -exec rm -rf {} + 2>/dev/null || true
