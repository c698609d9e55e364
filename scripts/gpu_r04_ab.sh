# Round-4 A/B: the headline bench (no aux lines) for the product library and each scripts/libgnsship_<V>.so
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r04ab
mkdir -p $O
for V in main ${VARIANTS:-}; do
  if [ $V = main ]; then LP=$R/gnss_sim_receiver_amd/libgnsship.so; else LP=$R/scripts/libgnsship_$V.so; fi
  GNSSHIP_LIB_PATH=$LP timeout -k 10 300 python -u bench.py --no-aux --cpu-seconds 0 > $O/bench_$V.json 2> $O/bench_$V.err || { echo "bench $V failed"; tail -20 $O/bench_$V.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$V.json'));print('variant $V value',d['value'],'us/epoch',d['us_per_epoch'])"
done
for V in ${TVARIANTS:-}; do
  if [ $V = main ]; then LP=$R/gnss_sim_receiver_amd/libgnsship.so; else LP=$R/scripts/libgnsship_$V.so; fi
  echo "timing $V"; GNSSHIP_LIB_PATH=$LP timeout -k 10 200 python3 scripts/trk_fast_timing.py 400 1 4 12 48 || { echo "timing $V failed"; exit 1; }
done
for PV in ${PVARIANTS:-}; do
  GNSSHIP_LIB_PATH=$R/scripts/libgnsship_$PV.so timeout -k 10 120 python3 scripts/trk_fast_profile.py 12 > $O/fast_phases_$PV.txt 2>&1 || { echo "profile $PV failed"; tail $O/fast_phases_$PV.txt; exit 1; }
  echo "---- profile $PV"; grep -v "HW_ID\|waves:\|states:" $O/fast_phases_$PV.txt
done
