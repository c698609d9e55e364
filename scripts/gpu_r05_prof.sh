# Round-5 phase timelines of trk_fast_kernel: full-stamp and group-stamp profiling builds.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05prof
mkdir -p $O
for v in ${VARIANTS:-xgrp xprof}; do
  GNSSHIP_LIB_PATH=$PWD/scripts/libgnsship_$v.so timeout -k 10 150 python3 scripts/trk_fast_profile.py 12 > $O/phases_$v.txt 2>&1 || { echo "profile $v failed"; tail $O/phases_$v.txt; exit 1; }
done
tail -n 60 $O/phases_*.txt
