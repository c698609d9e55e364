# A/B variants of the correlator (scripts/libgnsship_<tag>.so), selected with GNSSHIP_LIB_PATH.
#   bash scripts/build_variants.sh "w8:-DGNSSHIP_CORR_WAVES_EPL=8" "w6:-DGNSSHIP_CORR_WAVES_EPL=6"
set -e
cd "$(dirname "$0")/.."
make -s -j8 gnss_sim_receiver_amd/libgnsship.so
OBJS=$(ls build/obj/*.o | grep -v corr_kernel)
for spec in "$@"; do
  tag=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Iinclude -Ignss_sim_receiver_amd/csrc $flags \
    -c ${CORR_SRC:-gnss_sim_receiver_amd/csrc/corr_kernel.hip} -o build/corr_$tag.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o scripts/libgnsship_$tag.so $OBJS build/corr_$tag.o
  echo "built scripts/libgnsship_$tag.so"
done
