#!/bin/bash
# Links the objects scripts/build_variants.sh compiled: scripts/libgnsship_<name>.so
set -e
cd "$(dirname "$0")/.."
for name in "$@"; do
  VOBJ=$(ls build/var_$name/*.o)
  if [ "${PROF:-0}" = 1 ]; then OBJS=$(ls build/prof_obj/*.o | grep -v "/$(basename $VOBJ)$"); else OBJS=$(ls build/obj/*.o | grep -v "/$(basename $VOBJ)$"); fi
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o scripts/libgnsship_$name.so $OBJS $VOBJ -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
done
