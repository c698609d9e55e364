# Round-2: receiver / comm / tracking tests and the phase profile.  Stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r02rx
mkdir -p $O
timeout -k 10 120 python -u scripts/trk_wg_profile.py 1 12 sync > $O/phase.log 2>&1 || { echo "profile failed"; tail -20 $O/phase.log; exit 1; }
cat $O/phase.log
timeout -k 10 700 python -u -m pytest tests/test_gpu_comm.py tests/test_gpu_receiver.py tests/test_gpu_trk_persist.py tests/test_gpu_trk.py tests/test_gpu_reference_scenarios.py -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "PASS|FAIL|^E " $O/tests.log | head -60; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
echo "all ok"
