# the open-loop pipelined ring vs its split stages (bench's open_loop_correlator
# line with split_ms_per_launch), then the workgroup phase stamps of both launch forms.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/openloop
mkdir -p $O
timeout -k 10 200 python3 -u -c "
import json, torch, bench
from gnss_sim_receiver_amd import engine
ctx = engine.Context(0)
for rot in (0, 1, 0, 1):
    print(json.dumps(bench.open_loop_correlator(ctx, torch, 0, steps=60, rot=rot)), flush=True)
for rot in (0, 1):
    print(json.dumps(bench.e1_open_loop(ctx, rot=rot)), flush=True)
    print(json.dumps(bench.c5_open_loop(ctx, rot=rot)), flush=True)
" > $O/split.jsonl 2> $O/split.err || { echo "split failed"; tail -20 $O/split.err; exit 1; }
cat $O/split.jsonl
for mode in pipelined split; do
  GNSSHIP_LIB_PATH=$R/scripts/libgnsship_prof.so timeout -k 10 120 python3 scripts/corr_wg_profile.py $mode > $O/wg_$mode.txt 2>&1 || { echo "wg $mode failed"; tail $O/wg_$mode.txt; exit 1; }
  cat $O/wg_$mode.txt
done
echo "all ok"
