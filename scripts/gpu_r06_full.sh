# Round-6: the whole GPU suite, then the default bench line (both logged under gpurun_out/).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r06full}
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest -x -v -rA --timeout 170 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
  rc=$?
  tail -n 3 $O/tests.log
  [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/tests.log | head -20; exit 1; }
fi
timeout -k 10 900 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(json.dumps(d['summary']))"
exit 0
