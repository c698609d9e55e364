# Round-6 iteration: a chosen set of GPU tests (TESTS), one pytest process, then optionally the bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r06iter}
mkdir -p $O
timeout -k 10 ${TLIM:-900} python3 -u -m pytest -x -v -rA --timeout 170 --timeout-method thread -m gpu $TESTS > $O/tests.log 2>&1
rc=$?
tail -n 8 $O/tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error|assert" $O/tests.log | head -30; exit 1; }
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python3 bench.py $BENCH > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
  cat $O/bench.json
fi
exit 0
