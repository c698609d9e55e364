# Round-4 phase timeline of trk_fast_kernel (profiling build: scripts/libgnsship_prof.so) + headline bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r04prof
mkdir -p $O
timeout -k 10 120 python3 scripts/trk_fast_profile.py 12 > $O/fast_phases.txt 2>&1 || { echo "phase profile failed"; tail $O/fast_phases.txt; exit 1; }
cat $O/fast_phases.txt
