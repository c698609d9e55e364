# Iteration check on the GPU box: GPU tests (new ones first), default bench, 2-rank gloo rehearsal of
# the multi-rank bench on the one GPU.  Every GPU step has its own limit; stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/check
mkdir -p $O
FIRST=${FIRST:-}
if [ -n "$FIRST" ]; then
  timeout -k 10 300 python -u -m pytest $FIRST -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/first.log 2>&1 || { echo "first tests failed"; tail -40 $O/first.log; exit 1; }
fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
GNSSHIP_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --cpu-seconds 0 --no-acq > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err || { echo "n2 failed"; tail -20 $O/bench_n2_gloo.err; exit 1; }
cat $O/bench_n2_gloo.json
echo "all ok"
