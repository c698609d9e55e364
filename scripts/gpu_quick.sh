# Quick A/B on the GPU box: correlator parity tests, then the headline bench without the
# auxiliary legs.  Stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/quick
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_corr.py tests/test_gpu_corr_hd.py tests/test_gpu_e1.py -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 120 python bench.py --cpu-seconds 0 --no-acq > $O/bench$i.json 2> $O/bench$i.err || { echo "bench failed"; tail -20 $O/bench$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench$i.json'));print(d['value'],d['kernel_ms'],d['streaming_ibyte']['if_msamples_per_s'])"
done
