# Round-5 closing GPU suite (every -m gpu test, all failures listed).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r05final
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
