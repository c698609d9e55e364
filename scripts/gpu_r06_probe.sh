# Round-6 probes: the long-epoch closed-loop lines three times (variance of the E1 C4 share), the
# trk_fast phase timeline at GPS 25 Msps (12 channels), then the acquisition PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06probe
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 240 python3 -u scripts/long_epochs.py >> $O/long.txt 2>&1 || { tail -5 $O/long.txt; exit 1; }
done
cat $O/long.txt
timeout -k 10 240 python3 -u scripts/trk_fast_profile.py 12 25e6 > $O/phases_gps25.txt 2>&1 || { tail -5 $O/phases_gps25.txt; exit 1; }
head -12 $O/phases_gps25.txt
[ -n "$SKIP_PMC" ] && exit 0
bash scripts/gpu_acq_pmc.sh r06acq
