# Run the default bench line once per chunks-per-item setting (GNSSHIP_CHUNKS_PER_ITEM).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for k in "$@"; do
  GNSSHIP_CHUNKS_PER_ITEM=$k timeout -k 10 200 python bench.py --steps 20 --cpu-seconds 0 --no-acq > gpurun_out/abk_$k.json 2> gpurun_out/abk_$k.err || { echo "K=$k failed"; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/abk_$k.json')); print('K=$k', d['value'], d['kernel_ms'])"
done
