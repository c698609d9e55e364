# Round-4: instruction-cache counters of the headline kernel (one --pmc pass per group, kernel trace only).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r04ic
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -i "icache\|SQC_\|SQ_IFETCH\|SQ_WAIT_INST\|SQ_INSTS_VALU\b\|SQ_ACTIVE_INST" $O/avail.txt | head -60
cd $R
for C in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" "SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS"; do
  n=$(echo $C | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $C -d $O/pmc_$n -o pmc --output-format csv -- python3 bench.py --no-aux --steps 3 --warmup 1 --cpu-seconds 0 > $O/pmc_$n.log 2>&1 || { echo "pmc $n failed"; tail -5 $O/pmc_$n.log; }
done
python3 - <<'PY'
import csv, glob, os
O = os.environ.get("GRAFT_REPO_ROOT", ".") + "/gpurun_out/r04ic"
for f in sorted(glob.glob(O + "/pmc_*/**/*counter_collection.csv", recursive=True)):
    acc = {}
    for row in csv.DictReader(open(f)):
        if "trk_fast" not in row.get("Kernel_Name", ""):
            continue
        k = row["Counter_Name"]
        acc.setdefault(k, []).append(float(row["Counter_Value"]))
    for k, v in acc.items():
        print(f"{os.path.basename(os.path.dirname(f))}: {k} per launch {sum(v)/len(v):.4g} (launches {len(v)})")
PY
