# Round-6 E1 acquisition: A/B of a base build (scripts/libgnsship_base.so) against the current one,
# then the acquisition GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06acq
mkdir -p $O
L=gnss_sim_receiver_amd/libgnsship.so
timeout -k 10 200 python3 scripts/acq_e1_ab.py scripts/libgnsship_base.so $L > $O/ab.json 2>&1 || { tail -5 $O/ab.json; exit 1; }
cat $O/ab.json
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_acq.py tests/test_gpu_e1.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; exit $rc
