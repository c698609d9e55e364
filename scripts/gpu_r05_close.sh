# Round-5 last closing run: every -m gpu test, then the default bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r05close
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests.log | tail -12
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
