# Full round check on the GPU box: GPU tests, smoke(), default bench, rocprofv3 kernel stats of the
# bench, and the two PMC passes (FETCH_SIZE / WRITE_SIZE) for roofline.traffic.
# Each GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/full/pmc
O=$R/gpurun_out/full
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -30 $O/gpu_tests.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; cat $O/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 10 --warmup 2 --cpu-seconds 0 > $O/prof_bench.json 2> $O/prof_stderr.txt || { echo "rocprof failed"; exit 1; }
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/pmc/p$i -o run -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-acq > $O/pmc/p$i.json 2> $O/pmc_p$i.err || { echo "pmc pass $i failed"; exit 1; }
done
cd $R && python3 scripts/pmc_traffic.py $O/pmc > $O/pmc_summary.json && cat $O/pmc_summary.json
echo "all ok"
