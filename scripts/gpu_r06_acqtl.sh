# Round-6 E1 acquisition: A/B against the base build, and a kernel timeline of one sweep.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r06acqtl}
mkdir -p $O
L=gnss_sim_receiver_amd/libgnsship.so
timeout -k 10 200 python3 scripts/acq_e1_ab.py scripts/libgnsship_base.so $L > $O/ab.json 2>&1 || { tail -5 $O/ab.json; exit 1; }
cat $O/ab.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/tr -o run -- python3 $GRAFT_REPO_ROOT/scripts/acq_e1_ab.py --one > $GRAFT_REPO_ROOT/$O/tr.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/tr.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 scripts/acq_timeline.py $(find $O/tr -name "*kernel_trace.csv" | head -1) | tee $O/timeline.txt | tail -60
