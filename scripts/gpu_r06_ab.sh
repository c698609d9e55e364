# Round-6 A/B of trk_fast variants (scripts/libgnsship_<tag>.so; "base" = the product library):
# the headline bench line, ROUNDS passes over the variants in turn.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r06ab}
mkdir -p $O
for r in $(seq 1 ${ROUNDS:-2}); do
  for tag in "$@"; do
    lib=$PWD/scripts/libgnsship_$tag.so
    [ "$tag" = base ] && lib=$PWD/gnss_sim_receiver_amd/libgnsship.so
    GNSSHIP_LIB_PATH=$lib timeout -k 10 150 python3 bench.py --no-aux --cpu-seconds 0 --steps 20 --warmup 3 ${BENCH_ARGS:-} > $O/ab_${tag}_$r.json 2> $O/ab_${tag}_$r.err || { echo "variant $tag failed"; tail -3 $O/ab_${tag}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/ab_${tag}_$r.json')); print('$tag', $r, d['value'], d['us_per_epoch'])"
  done
done
exit 0
