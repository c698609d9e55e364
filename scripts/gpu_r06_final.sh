# Round-6 closing run: the default bench line, rocprofv3 kernel stats of the headline (bench --no-aux)
# and its PMC passes (FETCH_SIZE / WRITE_SIZE / SQ_INSTS_VALU, one group per pass, kernel trace
# only), the acquisition PMC passes (scripts/gpu_acq_pmc.sh) and the E1 sweep timeline.  Stops at the
# first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r06final
mkdir -p $O/pmc
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(json.dumps(d['summary']))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-aux --cpu-seconds 0 > $O/prof_bench.json 2> $O/prof_stderr.txt || { echo "rocprof failed"; tail $O/prof_stderr.txt; exit 1; }
i=0
for grp in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/pmc/p$i -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-aux --cpu-seconds 0 > $O/pmc/p$i.json 2> $O/pmc_p$i.err || { echo "pmc pass $i failed"; tail $O/pmc_p$i.err; exit 1; }
done
cd $R && python3 scripts/pmc_traffic.py $O/pmc trk_fast_kernel > $O/pmc_trk.json && head -12 $O/pmc_trk.json
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
find $O/pmc -mindepth 1 -type d -exec rm -rf {} + 2>/dev/null || true
find $O/prof -name "*kernel_trace.csv" -delete 2>/dev/null || true
bash scripts/gpu_acq_pmc.sh r06final_acq > $O/acq_pmc_out.txt 2>&1 || { echo "acq pmc failed"; tail $O/acq_pmc_out.txt; exit 1; }
OUT=r06final_tl bash scripts/gpu_r06_c3tl.sh > $O/c3tl_out.txt 2>&1 || { echo "c3 timeline failed"; tail $O/c3tl_out.txt; exit 1; }
echo "all ok"
