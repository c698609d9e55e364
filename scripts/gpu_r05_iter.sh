# Round-5 iteration: tracking-engine GPU tests (exact AVX paths), headline bench, phase profiles.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05iter
mkdir -p $O
T="${TESTS:-tests/test_gpu_headline_pin.py tests/test_gpu_trk_persist.py}"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu $T > $O/tests.log 2>&1
rc=$?
tail -n 5 $O/tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error" $O/tests.log | head -20; exit 1; }
timeout -k 10 200 python3 bench.py --no-aux --cpu-seconds 0 --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
for v in ${VARIANTS:-}; do
  GNSSHIP_LIB_PATH=$PWD/scripts/libgnsship_$v.so timeout -k 10 150 python3 scripts/trk_fast_profile.py 12 > $O/phases_$v.txt 2>&1 || { echo "profile $v failed"; tail $O/phases_$v.txt; exit 1; }
  grep -v "channel .*waves\|HW_ID" $O/phases_$v.txt
done
