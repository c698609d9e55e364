# Round-5 A/B: headline bench per library variant (scripts/libgnsship_<v>.so), then phase profiles.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ab
mkdir -p $O
for v in ${BVARIANTS:-}; do
  GNSSHIP_LIB_PATH=$PWD/scripts/libgnsship_$v.so timeout -k 10 150 python3 bench.py --no-aux --cpu-seconds 0 --steps 10 --warmup 2 > $O/bench_$v.json 2> $O/bench_$v.err || { echo "bench $v failed"; tail $O/bench_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/bench_$v.json')); print('$v', d['value'], d['us_per_epoch'])"
done
for v in ${VARIANTS:-}; do
  GNSSHIP_LIB_PATH=$PWD/scripts/libgnsship_$v.so timeout -k 10 150 python3 scripts/trk_fast_profile.py 12 > $O/phases_$v.txt 2>&1 || { echo "profile $v failed"; tail $O/phases_$v.txt; exit 1; }
  echo "== $v"; grep -E "epoch period|cycle:|tail:" $O/phases_$v.txt
done
if [ -n "${MAINBENCH:-}" ]; then
  timeout -k 10 150 python3 bench.py --no-aux --cpu-seconds 0 --steps 10 --warmup 2 > $O/bench_main.json 2> $O/bench_main.err || { echo "bench main failed"; tail $O/bench_main.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/bench_main.json')); print('main', d['value'], d['us_per_epoch'])"
fi
for v in ${LVARIANTS:-}; do
  if [ "$v" = main ]; then L=""; else L="GNSSHIP_LIB_PATH=$PWD/scripts/libgnsship_$v.so"; fi
  env $L timeout -k 10 200 python3 scripts/long_epochs.py ${LONGARGS:-} > $O/long_$v.txt 2>&1 || { echo "long $v failed"; tail $O/long_$v.txt; exit 1; }
  echo "== long $v"; grep -v amdgpu.ids $O/long_$v.txt
done
