# Round-6 trk_lane A/B: the 65536-channel sweep point (records) with the base and the current build,
# twice each interleaved, then the lane / throughput GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r06lane}
mkdir -p $O
for i in 1 2; do
  for L in ${LIBS:-scripts/libgnsship_base.so gnss_sim_receiver_amd/libgnsship.so}; do
    echo "$L" >> $O/ab.txt
    GNSSHIP_LIB_PATH=$PWD/$L timeout -k 10 240 python3 -u scripts/trk_sweep_point.py 65536 20 records >> $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
  done
done
grep -v amdgpu.ids $O/ab.txt
[ -n "$NO_TESTS" ] && exit 0
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 170 --timeout-method thread -m gpu tests/test_gpu_trk_lane.py tests/test_gpu_trk_thru.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; exit $rc
