# Round-6: C3 sweep timeline and host gaps (HIP API + kernel trace of scripts/acq_probe.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r06c3tl}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 180 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/tr -o run -- python3 $GRAFT_REPO_ROOT/scripts/acq_probe.py 10 > $GRAFT_REPO_ROOT/$O/tr.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/tr.log; exit 1; }
cd $GRAFT_REPO_ROOT
K=$(find $O/tr -name "*kernel_trace.csv" | head -1)
python3 scripts/acq_timeline.py $K "acq_fft_big_cols_kernel<0, 25>" > $O/c3_timeline.txt; cat $O/c3_timeline.txt
python3 scripts/acq_host_gaps.py $O/tr "search_big_kernel<25"
python3 scripts/acq_host_gaps.py $O/tr "acq_huge"
