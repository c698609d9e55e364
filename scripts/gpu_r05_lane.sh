# Round-5 trk_lane bring-up: the 1024-channel exact test, then sweep points (default dispatch vs
# trk_fast's throughput form).  Stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r05lane
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_trk_thru.py ${LANE_TESTS} > $O/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed|Error|assert" $O/tests.log | tail -20
[ $rc -eq 0 ] || exit 1
run() { echo "== $*" >> $O/sweep.txt; timeout -k 10 120 "$@" >> $O/sweep.txt 2>&1 || { echo "failed: $*"; tail -5 $O/sweep.txt; exit 1; }; }
run python3 scripts/trk_sweep_point.py 1024 20
run python3 scripts/trk_sweep_point.py 4096 20
run python3 scripts/trk_sweep_point.py 16384 20
run python3 scripts/trk_sweep_point.py 65536 20 records
grep -E "==|channels" $O/sweep.txt
