# Run the default bench line once per variant library (scripts/libgnsship_<tag>.so).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for tag in "$@"; do
  GNSSHIP_LIB_PATH=$R/scripts/libgnsship_$tag.so timeout -k 10 200 python bench.py --steps 20 --cpu-seconds 0 --no-acq > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || { echo "variant $tag failed"; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_$tag.json')); print('$tag', d['value'], d['kernel_ms'])"
done
