# Acquisition iteration: byte-for-byte A/B against the saved base library, the acquisition GPU tests,
# then the phase timeline of the C3 search kernel (profiling build).  Stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/acq_iter
mkdir -p $O
timeout -k 10 200 python3 scripts/acq_ab.py scripts/libgnsship_base.so gnss_sim_receiver_amd/libgnsship.so ${AB_FLAGS:-} > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt | tail -4
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "ab crashed rc=$rc"; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_acq.py tests/test_gpu_acq_resampler.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "acq tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python3 scripts/acq_wg_profile.py > $O/wg.txt 2>&1 || { echo "profile failed"; tail $O/wg.txt; exit 1; }
cat $O/wg.txt
echo "all ok"
