# Round-2 bench + profiles: default bench, rocprofv3 kernel stats of the headline (bench --no-aux),
# and the PMC passes (FETCH_SIZE / WRITE_SIZE / SQ_INSTS_VALU) of the headline kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r02bench
mkdir -p $O/pmc
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-aux > $O/prof_bench.json 2> $O/prof_stderr.txt || { echo "rocprof failed"; tail $O/prof_stderr.txt; exit 1; }
i=0
for grp in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/pmc/p$i -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-aux > $O/pmc/p$i.json 2> $O/pmc_p$i.err || { echo "pmc pass $i failed"; tail $O/pmc_p$i.err; exit 1; }
done
cd $R && python3 scripts/pmc_traffic.py $O/pmc trk_persist_kernel > $O/pmc_trk.json && cat $O/pmc_trk.json
find $O/prof -name "*kernel_stats.csv" | head -3

# acquisition kernels (C3 + C1 shape): kernel stats and PMC
bash $R/scripts/gpu_acq_pmc.sh acq || { echo "acq pmc failed"; exit 1; }
echo "all ok"
