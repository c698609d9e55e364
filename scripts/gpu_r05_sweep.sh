# Round-5 throughput end: sweep points through the default dispatch (trk_fast throughput form) and,
# for comparison, the persistent kernel (GNSSHIP_TRK_FAST=0).  SWEEP_ENV adds env (A/B); stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r05sweep
mkdir -p $O
run() { echo "== $*" >> $O/sweep.txt; timeout -k 10 120 env $SWEEP_ENV "$@" >> $O/sweep.txt 2>&1 || { echo "failed: $*"; tail -5 $O/sweep.txt; exit 1; }; }
run python3 scripts/trk_sweep_point.py 1024 20
run python3 scripts/trk_sweep_point.py 4096 20
run python3 scripts/trk_sweep_point.py 65536 20 records
GNSSHIP_TRK_FAST=0 run python3 scripts/trk_sweep_point.py 4096 20
GNSSHIP_TRK_FAST=0 run python3 scripts/trk_sweep_point.py 65536 20 records
cat $O/sweep.txt | grep -E "==|channels"
