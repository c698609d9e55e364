#!/bin/bash
# A/B builds of the fast tracking kernel: scripts/libgnsship_<name>.so = the product library with
# trk_fast.hip compiled under extra flags (the other objects are build/obj's).  Usage:
#   bash scripts/build_variants.sh name1 "-DX=1" name2 "-DY=2 -DZ=3" ...   [PROF=1: profiling builds]
# Then scripts/link_variants.sh name1 name2 ...   (SRC=trk_lane: vary trk_lane.hip instead)
set -e
cd "$(dirname "$0")/.."
make -s -j8 gnss_sim_receiver_amd/libgnsship.so
SRC=${SRC:-trk_fast}
BASE="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Iinclude -Ignss_sim_receiver_amd/csrc -Wall -Wno-unused-result"
[ "$SRC" = trk_fast ] && BASE="$BASE -fno-slp-vectorize"
if [ "${PROF:-0}" = 1 ]; then
  make -s -j8 prof
  BASE="$BASE -DGNSSHIP_CORR_PROFILE"
fi
pids=()
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  mkdir -p build/var_$name
  rm -f build/var_$name/*.o  # never link a stale object after a failed compile
  /opt/rocm/bin/hipcc $BASE $flags -c gnss_sim_receiver_amd/csrc/$SRC.hip -o build/var_$name/$SRC.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p" || { echo "a variant failed to compile" >&2; exit 1; }; done
