# Round-4 iteration: the trk_fast exactness tests, the phase timeline (profiling build), the headline bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r04iter
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline_pin.py tests/test_gpu_trk_persist.py tests/test_gpu_c5_closed_loop.py tests/test_gpu_trk.py -m gpu -q --timeout 280 --timeout-method thread ${PYTEST_K:-} > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|^ERROR|passed|failed|Error" $O/tests.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 120 python3 scripts/trk_fast_profile.py 12 > $O/fast_phases.txt 2>&1 || { echo "phase profile failed"; tail $O/fast_phases.txt; exit 1; }
cat $O/fast_phases.txt
timeout -k 10 300 python -u bench.py --no-aux --cpu-seconds 0 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('value',d['value'],'us/epoch',d['us_per_epoch'])"
for V in ${VARIANTS:-}; do
  GNSSHIP_LIB_PATH=$R/scripts/libgnsship_$V.so timeout -k 10 300 python -u bench.py --no-aux --cpu-seconds 0 > $O/bench_$V.json 2> $O/bench_$V.err || { echo "bench $V failed"; tail -20 $O/bench_$V.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$V.json'));print('variant $V value',d['value'],'us/epoch',d['us_per_epoch'])"
done
for PV in ${PVARIANTS:-}; do
  GNSSHIP_LIB_PATH=$R/scripts/libgnsship_$PV.so timeout -k 10 120 python3 scripts/trk_fast_profile.py 12 > $O/fast_phases_$PV.txt 2>&1 || { echo "profile $PV failed"; tail $O/fast_phases_$PV.txt; exit 1; }
  echo "---- profile $PV"; grep -E "epoch period|group . seen|group . ready" $O/fast_phases_$PV.txt
done
