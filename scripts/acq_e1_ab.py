"""A/B of the Galileo E1 all-sky search (32 PRN x 40 bins, N = 100000 at 25 Msps, the huge layout)
between two builds, each in its own process (GNSSHIP_LIB_PATH): per-PRN Doppler / code index /
statistic and the sweep time.
    python scripts/acq_e1_ab.py scripts/libgnsship_base.so gnss_sim_receiver_amd/libgnsship.so
Either side may carry environment settings after a colon: lib.so:GNSSHIP_ACQ_LANES=1,OTHER=2."""
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_one():
    sys.path.insert(0, ROOT)
    from gnss_sim_receiver_amd import codes as C, engine, signals as S
    ctx = engine.Context(0)
    fs, n = 25000000, 100000
    sats = S.random_sky(6, seed=0x6E550002 + 7, system="GAL", prns=[2, 9, 13, 21, 26, 31])
    sig = S.generate_if(fs, n, sats, seed=0x6E550002 + 7)
    acq = engine.PcpsAcquisition(ctx, fs, n, 5000, 250, 0, False, max_prns=32, ms_per_code=4)
    for k in range(32):
        acq.set_local_code(C.galileo_e1_code_gen_complex_sampled("1B", False, k + 1, fs), k)
    dev = ctx.upload(np.ascontiguousarray(sig))
    for _ in range(2):
        acq.run(dev, n_prns=32)
    t0 = time.perf_counter()
    reps = 30
    for _ in range(reps):
        res, _ = acq.run(dev, n_prns=32)
    dt = (time.perf_counter() - t0) / reps
    out = {"sweep_ms": dt * 1e3, "rows": [[r.doppler_index, r.code_index, float(r.test_statistic), float(r.peak)] for r in res]}
    print("RESULT " + json.dumps(out), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--one":
        run_one()
        return
    outs = []
    runs = []
    for spec in sys.argv[1:3] * 2:  # A, B, A, B: each side's best of two processes
        lib, _, extra = spec.partition(":")
        env = dict(os.environ, GNSSHIP_LIB_PATH=os.path.abspath(lib))
        env.update(kv.split("=", 1) for kv in extra.split(",") if kv)
        p = subprocess.run([sys.executable, os.path.abspath(__file__), "--one"], env=env, capture_output=True, text=True, timeout=300)
        line = [x for x in p.stdout.splitlines() if x.startswith("RESULT ")]
        if not line:
            print(p.stdout[-2000:], p.stderr[-2000:])
            raise SystemExit(f"{lib}: no result")
        runs.append(json.loads(line[0][7:]))
    for k in range(2):
        best = min((runs[k], runs[k + 2]), key=lambda o: o["sweep_ms"])
        outs.append(best)
    a, b = outs
    same_idx = sum(1 for x, y in zip(a["rows"], b["rows"]) if x[0] == y[0] and x[1] == y[1])
    dstat = max(abs(x[2] - y[2]) / max(abs(x[2]), 1e-30) for x, y in zip(a["rows"], b["rows"]))
    dpeak = max(abs(x[3] - y[3]) / max(abs(x[3]), 1e-30) for x, y in zip(a["rows"], b["rows"]))
    print(json.dumps({"base_sweep_ms": round(a["sweep_ms"], 3), "new_sweep_ms": round(b["sweep_ms"], 3), "prns_same_doppler_and_index": same_idx,
                      "max_rel_stat_diff": dstat, "max_rel_peak_diff": dpeak,
                      "diffs": [(k + 1, x, y) for k, (x, y) in enumerate(zip(a["rows"], b["rows"])) if x[:2] != y[:2]]}))


if __name__ == "__main__":
    main()
