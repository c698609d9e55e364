set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof_iter
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -q -rf > gpurun_out/gpu_tests.log 2>&1; echo "pytest rc=$?" >> gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/bench_iter.json 2> gpurun_out/bench_iter.err && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_iter -o run -- python3 $R/bench.py --steps 10 --warmup 2 --cpu-seconds 0 > $R/gpurun_out/prof_iter/bench.json 2> $R/gpurun_out/prof_iter/stderr.txt
echo "all rc=$?"
