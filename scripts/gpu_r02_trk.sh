# Round-2 closed-loop check: new persistent-loop tests first, then the existing tracking tests,
# then the timing probe.  Every GPU step has its own limit; stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r02trk
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_trk_persist.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/persist_tests.log 2>&1 || { echo "persist tests failed"; tail -60 $O/persist_tests.log; exit 1; }
tail -3 $O/persist_tests.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_trk.py tests/test_gpu_reference_scenarios.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/trk_tests.log 2>&1 || { echo "trk tests failed"; tail -60 $O/trk_tests.log; exit 1; }
tail -3 $O/trk_tests.log
timeout -k 10 300 python -u scripts/trk_probe.py > $O/probe.log 2>&1 || { echo "probe failed"; tail -30 $O/probe.log; exit 1; }
cat $O/probe.log
echo "all ok"
