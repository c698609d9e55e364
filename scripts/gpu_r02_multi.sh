# Round-2: tests of the comm / sharded paths and the closed loop, the phase profile, the default
# bench (N=1), and a two-rank rehearsal of the multi-GPU flow on the one-GPU box (gloo; RCCL refuses
# two ranks on one device, so the C-ABI communicator reports its failure and the fan-out falls back).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r02multi
mkdir -p $O
timeout -k 10 120 python -u scripts/trk_wg_profile.py 1 12 sync > $O/phase.log 2>&1 || { echo "profile failed"; tail -20 $O/phase.log; exit 1; }
cat $O/phase.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_comm.py tests/test_gpu_trk_persist.py tests/test_gpu_trk.py tests/test_gpu_reference_scenarios.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
GNSSHIP_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --cpu-seconds 0 --sharded-aux-only > $O/bench_n2.json 2> $O/bench_n2.err || { echo "n2 rehearsal failed"; tail -30 $O/bench_n2.err; exit 1; }
cat $O/bench_n2.json
echo "all ok"
