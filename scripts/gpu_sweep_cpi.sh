# Sweep GNSSHIP_CHUNKS_PER_ITEM (work-item size of the correlator) on the headline bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/sweep
mkdir -p $O
for c in 1 2 3 4; do
  GNSSHIP_CHUNKS_PER_ITEM=$c timeout -k 10 120 python bench.py --cpu-seconds 0 --no-acq > $O/cpi$c.json 2> $O/cpi$c.err || { echo "bench failed"; tail -20 $O/cpi$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/cpi$c.json'));print('cpi $c', d['value'],d['kernel_ms'])"
done
