set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/trace
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace -o run -- python3 $R/bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-acq > $R/gpurun_out/trace/bench.json 2> $R/gpurun_out/trace/err.txt
echo rc=$?
