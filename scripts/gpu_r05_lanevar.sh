# trk_lane A/B: sweep points per variant library (LIBS: names of scripts/libgnsship_<name>.so; "main" = the product build).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r05lane
mkdir -p $O
for v in ${LIBS:-main}; do
  if [ "$v" = main ]; then LP=$R/gnss_sim_receiver_amd/libgnsship.so; else LP=$R/scripts/libgnsship_$v.so; fi
  for pt in ${PTS:-1024 4096 65536}; do
    echo "== $v $pt" >> $O/var.txt
    GNSSHIP_LIB_PATH=$LP timeout -k 10 120 python3 scripts/trk_sweep_point.py $pt 20 >> $O/var.txt 2>&1 || { echo "failed $v $pt"; tail -5 $O/var.txt; exit 1; }
  done
done
grep -E "==|channels" $O/var.txt | sed 's/kernel trk_lane_kernel.*records/records/'
