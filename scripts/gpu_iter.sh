# Iteration run on the GPU box: GPU tests, default bench, rocprofv3 kernel stats of a short bench.
# Stops at the first crash / signal / timeout (pytest rc other than 0 or 1).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof_iter
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -q -rf > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench_iter.json 2> gpurun_out/bench_iter.err && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_iter -o run -- python3 $R/bench.py --steps 10 --warmup 2 --cpu-seconds 0 > $R/gpurun_out/prof_iter/bench.json 2> $R/gpurun_out/prof_iter/stderr.txt
echo "all rc=$?"
