# Round-3 profiles: rocprofv3 kernel stats of the headline (bench --no-aux: trk_fast_kernel), its PMC
# passes (FETCH_SIZE / WRITE_SIZE / SQ_INSTS_VALU, one group per pass), then the acquisition kernels'
# stats and PMC (scripts/gpu_acq_pmc.sh).  Stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03prof
mkdir -p $O/pmc
cd $R && timeout -k 10 200 python -u -m pytest tests/test_gpu_receiver.py -m gpu -q --timeout 150 --timeout-method thread > $O/rx_tests.log 2>&1; echo "rx tests rc=$?"; tail -2 $O/rx_tests.log
timeout -k 10 120 python3 scripts/trk_fast_profile.py 12 > $O/fast_phases.txt 2>&1 || { echo "phase profile failed"; tail $O/fast_phases.txt; exit 1; }
cat $O/fast_phases.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-aux --cpu-seconds 0 > $O/prof_bench.json 2> $O/prof_stderr.txt || { echo "rocprof failed"; tail $O/prof_stderr.txt; exit 1; }
cat $O/prof_bench.json
i=0
for grp in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/pmc/p$i -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-aux --cpu-seconds 0 > $O/pmc/p$i.json 2> $O/pmc_p$i.err || { echo "pmc pass $i failed"; tail $O/pmc_p$i.err; exit 1; }
done
cd $R && python3 scripts/pmc_traffic.py $O/pmc trk_fast_kernel > $O/pmc_trk.json && cat $O/pmc_trk.json
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
find $O/pmc -mindepth 1 -type d -exec rm -rf {} + 2>/dev/null || true
bash $R/scripts/gpu_acq_pmc.sh r03acq || { echo "acq pmc failed"; exit 1; }
find $R/gpurun_out/pmc_r03acq -mindepth 1 -type d -exec rm -rf {} + 2>/dev/null || true
echo "all ok"
