# Iteration: the tracking and acquisition GPU tests, the E1 all-sky A/B (one batch lane vs two),
# then the headline bench line.  Stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/iter2
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_trk.py tests/test_gpu_trk_persist.py tests/test_gpu_headline_pin.py tests/test_gpu_c5_closed_loop.py tests/test_gpu_receiver.py tests/test_gpu_reference_scenarios.py tests/test_gpu_acq.py tests/test_gpu_acq_resampler.py -m gpu -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $O/tests.log | tail -2; grep -E "^FAILED" $O/tests.log | head -10
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
L=gnss_sim_receiver_amd/libgnsship.so
timeout -k 10 300 python3 scripts/acq_e1_ab.py $L:GNSSHIP_ACQ_LANES=1 $L > $O/e1_ab.txt 2>&1 || { echo "e1 ab failed"; tail $O/e1_ab.txt; exit 1; }
cat $O/e1_ab.txt
timeout -k 10 300 python3 scripts/acq_e1_ab.py $L:GNSSHIP_ACQ_LANES=2,GNSSHIP_ACQ_U_MIB=256 $L > $O/e1_ab256.txt 2>&1 || { echo "e1 ab 256 failed"; tail $O/e1_ab256.txt; exit 1; }
cat $O/e1_ab256.txt
timeout -k 10 300 python3 bench.py --no-aux --cpu-seconds 0 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
cat $O/bench.json
