# Full GPU check: the GPU suite (no -x: every failure is listed), the C1 receiver test on the
# trk_persist path for comparison, then the default bench line.
set -o pipefail
mkdir -p gpurun_out/r03a
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r03a/gpu_tests.log 2>&1
rc=$?
echo "suite rc=$rc"; tail -8 gpurun_out/r03a/gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
GNSSHIP_TRK_FAST=0 timeout -k 10 200 python -u -m pytest tests/test_gpu_receiver.py -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/r03a/rx_persist.log 2>&1
echo "persist rx rc=$?"; tail -4 gpurun_out/r03a/rx_persist.log
timeout -k 10 400 python -u bench.py > gpurun_out/r03a/bench.json 2> gpurun_out/r03a/bench.err || { echo bench failed; tail -20 gpurun_out/r03a/bench.err; exit 1; }
cat gpurun_out/r03a/bench.json
