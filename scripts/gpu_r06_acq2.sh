# Round-6 E1 acquisition: U budget / lane A/B and a kernel-stats profile of the sweeps.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r06acq2}
mkdir -p $O
L=gnss_sim_receiver_amd/libgnsship.so
for v in ${VARS:-GNSSHIP_ACQ_U_MIB=256 GNSSHIP_ACQ_U_MIB=64 GNSSHIP_ACQ_LANES=1 GNSSHIP_ACQ_U_MIB=384}; do
  echo "$v" >> $O/ab.txt
  timeout -k 10 200 python3 scripts/acq_e1_ab.py $L $L:$v >> $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
done
cat $O/ab.txt
[ -n "$NO_STATS" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/stats -o run -- python3 $GRAFT_REPO_ROOT/scripts/acq_probe.py 10 > $GRAFT_REPO_ROOT/$O/stats.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/stats.log; exit 1; }
cd $GRAFT_REPO_ROOT && find $O/stats -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \; && tail -3 $O/stats.log
