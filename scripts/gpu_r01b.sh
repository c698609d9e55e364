# Round-1 check: GPU tests (incl. C++ mirror), N=1 bench, 2-rank rehearsal over gloo on one GPU.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -rf > gpurun_out/gpu_tests.log 2>&1; echo "pytest rc=$?" >> gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --cpu-seconds 5 > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || { echo "bench n1 failed"; exit 1; }
GNSSHIP_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 > gpurun_out/bench_n2_gloo.json 2> gpurun_out/bench_n2_gloo.err
echo "n2 rc=$?"
