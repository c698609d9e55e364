# Tracking iteration: the tracking GPU tests (closed loops, the headline pin, C5, the receiver), the
# fast kernel's phase timeline (profiling build; and the LDS-parameter variant), and the headline
# bench line.  Stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/trk_iter
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_trk.py tests/test_gpu_trk_persist.py tests/test_gpu_headline_pin.py tests/test_gpu_c5_closed_loop.py tests/test_gpu_receiver.py tests/test_gpu_reference_scenarios.py -m gpu -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $O/tests.log | tail -3; grep -E "^FAILED|Error" $O/tests.log | head -10
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 120 python3 scripts/trk_fast_profile.py 12 > $O/fast_phases.txt 2>&1 || { echo "phase profile failed"; tail $O/fast_phases.txt; exit 1; }
cat $O/fast_phases.txt
if [ -f scripts/libgnsship_ldsk.so ]; then
GNSSHIP_LIB_PATH=$R/scripts/libgnsship_ldsk.so timeout -k 10 120 python3 scripts/trk_fast_profile.py 12 > $O/fast_phases_ldsk.txt 2>&1 || { echo "phase profile ldsk failed"; exit 1; }
head -24 $O/fast_phases_ldsk.txt
fi
timeout -k 10 300 python3 bench.py --no-aux --cpu-seconds 0 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
cat $O/bench.json
