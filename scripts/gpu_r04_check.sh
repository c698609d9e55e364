# Round-4 check: the GPU suite (all failures listed; stops the call on a crash), then the headline
# bench line alone.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r04check
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $O/gpu_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests.log | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python -u bench.py --no-aux --cpu-seconds 0 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
