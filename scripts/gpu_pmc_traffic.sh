# HBM traffic of the dominant kernel (corr_batch_kernel) for bench.py's roofline.traffic:
# two separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE), kernel-trace only, then
# scripts/pmc_traffic.py → profiles/pmc_corr.json (MI355X_MICROARCH.md §HBM corrections).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_traffic
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --cpu-seconds 0 --no-acq"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py $ARGS > $OUT/p$i.json 2> $OUT/p$i.err || { echo "pass $i failed rc=$?"; exit 1; }
done
cd $R && python3 scripts/pmc_traffic.py $OUT > $OUT/summary.json && cat $OUT/summary.json
