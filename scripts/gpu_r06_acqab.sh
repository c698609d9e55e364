# Round-6 acquisition A/B (C3, C1 shape, E1; results byte for byte) against scripts/libgnsship_base.so,
# then the acquisition GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r06acqab}
mkdir -p $O
timeout -k 10 300 python3 scripts/acq_ab.py scripts/libgnsship_base.so gnss_sim_receiver_amd/libgnsship.so $AB_FLAGS > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_acq.py tests/test_gpu_e1.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; exit $rc
