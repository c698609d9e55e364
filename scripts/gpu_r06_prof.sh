# Round-6: the fast kernel's phase timeline (profiling build) and the headline bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r06prof}
mkdir -p $O
timeout -k 10 200 python3 bench.py --no-aux --cpu-seconds 0 --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('value', d['value'], 'us/epoch', d['us_per_epoch'])"
GNSSHIP_LIB_PATH=$PWD/scripts/libgnsship_prof.so timeout -k 10 150 python3 scripts/trk_fast_profile.py 12 > $O/phases.txt 2>&1 || { echo "profile failed"; tail $O/phases.txt; exit 1; }
grep -v "channel .*waves\|HW_ID" $O/phases.txt
exit 0
