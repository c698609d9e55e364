# Dynamic instruction mix of the bench's kernels: two PMC passes (--kernel-trace only).
#   bash scripts/gpu_pmc_inst.sh <tag>   (library scripts/libgnsship_<tag>.so, or the default one if tag=default)
set -o pipefail
R=$GRAFT_REPO_ROOT
tag=${1:-default}
OUT=$R/gpurun_out/pmci_$tag
mkdir -p $OUT
[ "$tag" != default ] && export GNSSHIP_LIB_PATH=$R/scripts/libgnsship_$tag.so
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --cpu-seconds 0 --no-acq"
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" "SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py $ARGS > $OUT/p$i.json 2> $OUT/p$i.err || { echo "pass $i failed rc=$?"; exit 1; }
done
cd $R && python scripts/pmc_summary.py $OUT > $OUT/summary.json && echo "pmc $tag done"
