# Replay-chain probe: the isolated replay microbenchmark (with idle / polling / VALU-busy neighbour
# waves, with and without s_setprio), then the fast kernel's phase timeline, base and with the replay
# wave at priority 3 (profiling builds).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/replay_probe
mkdir -p $O
timeout -k 10 60 ./scripts/replay_bench > $O/replay_bench.txt 2>&1 || { echo "replay bench failed"; cat $O/replay_bench.txt; exit 1; }
cat $O/replay_bench.txt
timeout -k 10 120 python3 scripts/trk_fast_profile.py 12 > $O/fast_phases.txt 2>&1 || { echo "phase profile failed"; tail $O/fast_phases.txt; exit 1; }
head -9 $O/fast_phases.txt; grep "replay  " $O/fast_phases.txt
GNSSHIP_LIB_PATH=$R/scripts/libgnsship_prio.so timeout -k 10 120 python3 scripts/trk_fast_profile.py 12 > $O/fast_phases_prio.txt 2>&1 || { echo "phase profile prio failed"; exit 1; }
head -9 $O/fast_phases_prio.txt; grep "replay  " $O/fast_phases_prio.txt
