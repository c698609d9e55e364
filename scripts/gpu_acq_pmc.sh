# Acquisition kernels: rocprofv3 kernel stats and PMC passes (SQ instruction mix / stalls / LDS bank
# conflicts; FETCH_SIZE and WRITE_SIZE in separate passes), summarised by scripts/pmc_summary.py.
set -o pipefail
R=$GRAFT_REPO_ROOT
tag=${1:-acq}
OUT=$R/gpurun_out/pmc_$tag
mkdir -p $OUT
cd $R && timeout -k 10 120 python3 scripts/acq_probe.py 20 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 $R/scripts/acq_probe.py 10 > $OUT/stats.log 2>&1 || { echo "stats failed"; tail -5 $OUT/stats.log; exit 1; }
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 $R/scripts/acq_probe.py 3 > $OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 $OUT/p$i.log; exit 1; }
done
cd $R && python3 scripts/pmc_summary.py $OUT > $OUT/summary.json && python3 -c "
import json; d=json.load(open('$OUT/summary.json'))
for k,v in d.items():
    if 'acq' in k: print(k, {a: round(b) for a,b in v.items()})
"
find $OUT/stats -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
grep -i acq $OUT/kernel_stats.csv | cut -c1-200
echo "all ok"
