# Run GPU tests against a variant library (GNSSHIP_LIB_PATH): LIB=<variant> TESTS="..."
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05iter
mkdir -p $O
GNSSHIP_LIB_PATH=$PWD/scripts/libgnsship_$LIB.so timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu $TESTS > $O/tests_$LIB.log 2>&1
rc=$?
tail -n 3 $O/tests_$LIB.log
exit $rc
