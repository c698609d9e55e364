# Round-5 bench line: the default bench.py run (every auxiliary line), then the long-epoch lines alone.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r05bench
mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], d["unit"], "ms/step", d["ms_per_step"], "roofline", d.get("roofline", {}).get("frac"))
print("cpu_baseline", d.get("cpu_baseline", {}).get("value"))
print("sustained", d.get("tracked_channels_sustained"))
for r in d.get("channel_sweep", []):
    print("  sweep", r["channels"], r["kernel"][:22], r["realtime_factor"], r["kernel_us_per_round"], r["us_per_epoch_round"])
for k in ("closed_loop_gps_25msps", "closed_loop_e1_25msps_c4_share", "closed_loop_c5_share", "closed_loop_c4_full_64_e1", "closed_loop_c5_full_256"):
    v = d.get(k, {})
    print(k, v.get("realtime_factor"), v.get("us_per_epoch_round"))
for k in ("acquisition_c3", "acquisition_e1", "acquisition"):
    v = d.get(k, {})
    print(k, {f: v.get(f) for f in ("ms_per_sweep", "sweeps_per_s", "present_min_test_statistic", "absent_max_test_statistic", "roofline_frac") if f in v})
PY
