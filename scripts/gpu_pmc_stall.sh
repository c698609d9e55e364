# Where the correlator's wave cycles go: SQ stall/active buckets and the dynamic instruction mix,
# two PMC passes (--kernel-trace only), summarised per kernel by scripts/pmc_summary.py.
set -o pipefail
R=$GRAFT_REPO_ROOT
tag=${1:-default}
OUT=$R/gpurun_out/pmcs_$tag
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --cpu-seconds 0 --no-acq"
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py $ARGS > $OUT/p$i.json 2> $OUT/p$i.err || { echo "pass $i failed rc=$?"; tail -5 $OUT/p$i.err; exit 1; }
done
cd $R && python3 scripts/pmc_summary.py $OUT > $OUT/summary.json && python3 -c "
import json; d=json.load(open('$OUT/summary.json'))
for k,v in d.items():
    if 'corr_batch' in k or 'anchor' in k: print(k, {a: round(b) for a,b in v.items()})
"
