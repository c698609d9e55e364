# Round-6: host gaps of the E1 and C3 sweeps (HIP API + kernel trace).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r06hostgap}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 120 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/e1 -o run -- python3 $GRAFT_REPO_ROOT/scripts/acq_e1_ab.py --one > $GRAFT_REPO_ROOT/$O/e1.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/e1.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 scripts/acq_host_gaps.py $O/e1
